#!/bin/bash
# C5 SpMV: sparse GPU tests, fp64 / fp32 bench lines, PMC passes of both arms (tools/pmc_summary_spmv.py)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/c5pmc
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_default_path.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --config c5 > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
timeout -k 10 300 python bench.py --config c5 --f32 > $O/bench_c5_f32.json 2> $O/bench_c5_f32.err || exit 1
run() {  # arm, name, counters...
  local arm=$1 name=$2; shift 2
  local fl=""; [ $arm = f32 ] && fl="--f32"
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$arm/$name -o $name -- python3 bench.py --config c5 $fl --steps 1 --warmup 0 --no-cpu-baseline --no-check > $O/$arm/$name.log 2>&1
  local rc=$?; echo "pmc $arm $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
for arm in f64 f32; do
  mkdir -p $O/$arm
  run $arm fetch FETCH_SIZE
  run $arm write WRITE_SIZE
  run $arm tcc TCC_HIT_sum TCC_MISS_sum
done
echo done
