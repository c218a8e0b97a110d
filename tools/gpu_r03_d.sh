#!/bin/bash
# r03: the Cholesky chain as dependency-driven launches -- bitwise parity vs one launch per
# operation and vs the serial order, then c2 (and the c3 shape) under rocprofv3 with SCS_CHOL_DAG 0/1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread \
  "tests/test_gpu_parity.py::test_cholesky_dag_launches_bit_identical" \
  "tests/test_gpu_parity.py::test_cholesky_lookahead_bit_identical" "tests/test_gpu_parity.py::test_cholesky_diag_pipe_bit_identical" \
  "tests/test_gpu_parity.py::test_blocked_cholesky_solve" "tests/test_gpu_default_path.py::test_default_path_newton_methods" \
  "tests/test_gpu_default_path.py::test_c4_shape_solve_backward_error" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for dg in 0 1; do
  SCS_CHOL_DAG=$dg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_c2_dag$dg -o run -- python3 bench.py \
    --config c2 --steps 3 --warmup 1 --no-cpu-baseline > $O/c2_dag$dg.log 2>&1 || { echo "c2 dag$dg failed"; tail -5 $O/c2_dag$dg.log; exit 1; }
  grep '^{' $O/c2_dag$dg.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 dag=$dg', round(d['value'],4), 'solve_ms', round(d['breakdown_ms_per_step']['solve'],3))"
  python3 tools/rocpd_stats.py $O/rp_c2_dag$dg/run_results.db --csv $O/c2_dag$dg.csv > /dev/null
done
for dg in 0 1; do
  SCS_CHOL_DAG=$dg timeout -k 10 300 python3 bench.py --config c3 --N 131072 --steps 3 --warmup 1 --no-cpu-baseline \
    > $O/c3_dag$dg.json 2> $O/c3_dag$dg.err || { echo "c3 dag$dg failed"; tail -3 $O/c3_dag$dg.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_dag$dg.json').read().strip().splitlines()[-1]); print('c3 dag=$dg', round(d['value'],4), 'solve_ms', round(d['breakdown_ms_per_step']['solve'],3))"
done
