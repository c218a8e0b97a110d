#!/bin/bash
# r03: one-launch triangular solves (register-prefetched tiles, butterfly column GEMV) -- parity,
# then c2 / c3-shape bench with SCS_SOLVE_PERSIST 0/1 under rocprofv3 kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread \
  "tests/test_gpu_parity.py::test_one_launch_triangular_solves" "tests/test_gpu_parity.py::test_blocked_cholesky_solve" \
  "tests/test_gpu_default_path.py::test_default_path_newton_methods" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for ps in 0 1; do
  SCS_SOLVE_PERSIST=$ps timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_c2_ps$ps -o run -- python3 bench.py \
    --config c2 --steps 3 --warmup 1 --no-cpu-baseline > $O/c2_ps$ps.log 2>&1 || { echo "c2 ps$ps failed"; tail -5 $O/c2_ps$ps.log; exit 1; }
  grep '^{' $O/c2_ps$ps.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 persist=$ps', round(d['value'],4), 'solve_ms', round(d['breakdown_ms_per_step']['solve'],3))"
  python3 tools/rocpd_stats.py $O/rp_c2_ps$ps/run_results.db --csv $O/c2_ps$ps.csv | grep -E "persist|fwd|bwd|chol_diag|gram_small" | cut -c1-60,200-
done
