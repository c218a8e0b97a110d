#!/bin/bash
# r03: C5 fp32-vs-fp64 tolerance study at full size, then the default-config profile run that used to
# fault at exit (CU-masked bulk stream now off by default): rocprofv3 kernel-trace stats of c2 and c3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_multi.py \
  "tests/test_gpu_parity.py::test_one_launch_triangular_solves" "tests/test_gpu_parity.py::test_blocked_cholesky_solve" \
  "tests/test_gpu_default_path.py::test_default_path_newton_methods" "tests/test_gpu_default_path.py::test_c4_shape_solve_backward_error" \
  > $O/pytest_multi.log 2>&1
rc=$?; echo "pytest multi rc=$rc"; tail -3 $O/pytest_multi.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u tools/c5_tolerance.py --out $O/tolerance.json > $O/tol.log 2>&1
rc=$?; echo "tolerance rc=$rc"; tail -3 $O/tol.log; [ $rc -eq 0 ] || exit $rc
for cfg in c2 c3; do
  extra=""; [ $cfg = c3 ] && extra="--N 131072"
  for ps in 0 1; do
    SCS_SOLVE_PERSIST=$ps timeout -k 10 300 python3 bench.py --config $cfg $extra --steps 3 --warmup 1 --no-cpu-baseline \
      > $O/${cfg}_ps$ps.json 2> $O/${cfg}_ps$ps.err || { echo "bench $cfg failed"; tail -3 $O/${cfg}_ps$ps.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${cfg}_ps$ps.json').read().strip().splitlines()[-1]); print('$cfg persist=$ps', round(d['value'],4), 'solve_ms', round(d['breakdown_ms_per_step']['solve'],3), d.get('parity_check',{}).get('pass'))"
  done
done
SCS_SEGV_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_c2 -o run -- python3 bench.py --config c2 \
  --steps 3 --warmup 1 --no-cpu-baseline --no-check > $O/prof_c2.log 2>&1
rc=$?; echo "rocprofv3 default c2: exit $rc"; tail -c 600 $O/prof_c2.log; [ $rc -eq 0 ] || exit $rc
