#!/bin/bash
# r03 first call: the new parity tests (∇fx, C4-shape GGN + gl, gl / rebatch shards), the bench
# launcher (--gpus 2 on one GPU with --share-device; --gpus 8 must refuse), then the exit-time fault
# under rocprofv3 with the default (CU-masked) bulk stream, with SCS_SEGV_TRACE naming the frames
# (last: a crash ends the call).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 900 --timeout-method thread \
  "tests/test_gpu_parity.py::test_step_grad_fx_keyword" tests/test_gpu_shard.py \
  "tests/test_gpu_default_path.py::test_c4_shape_ggn_group_lasso" tests/test_gpu_sparse.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 2 --comm torch --share-device --N 131072 --steps 3 --warmup 1 \
  --no-cpu-baseline > $O/bench_g2.json 2> $O/bench_g2.err
rc=$?; echo "bench --gpus 2 rc=$rc"; tail -c 1500 $O/bench_g2.json; [ $rc -eq 0 ] || { tail -5 $O/bench_g2.err; exit $rc; }
timeout -k 10 120 python3 bench.py --gpus 8 > $O/bench_g8.json 2> $O/bench_g8.err
echo "bench --gpus 8 on one GPU: rc=$? (expected non-zero)"; tail -2 $O/bench_g8.err
timeout -k 10 600 python3 bench.py --config c5ggn --steps 2 --warmup 0 --no-cpu-baseline --no-check \
  > $O/bench_c5ggn.json 2> $O/bench_c5ggn.err
rc=$?; echo "bench c5ggn rc=$rc"; tail -c 2500 $O/bench_c5ggn.json; [ $rc -eq 0 ] || { tail -5 $O/bench_c5ggn.err; exit $rc; }
SCS_SEGV_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp -o run -- python3 bench.py --config c2 \
  --steps 1 --warmup 0 --no-cpu-baseline --no-check > $O/prof.log 2>&1
echo "rocprofv3 default c2: exit $?"; grep -A40 "\[scsopt\] signal" $O/prof.log | head -50
