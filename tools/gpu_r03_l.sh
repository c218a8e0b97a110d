#!/bin/bash
# r03: reference-solver QR speed -- QR tests, wall time at m = 2048 / 8192, kernel stats of the m = 8192 solve.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03l; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_gpu_parity.py::test_householder_qr_solve" "tests/test_gpu_parity.py::test_reference_solver_trajectory" \
  "tests/test_gpu_parity.py::test_reference_solver_ill_conditioned" > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/qr_time.py 2048 8192 > $O/qr_time.log 2>&1; rc=$?; echo "qr timing rc=$rc"; grep "m=" $O/qr_time.log; [ $rc -eq 0 ] || exit $rc
SCS_QR_STEP=0 timeout -k 10 300 python3 tools/qr_time.py 8192 > $O/qr_time_3launch.log 2>&1; rc=$?; echo "qr timing (3 launches per column) rc=$rc"; grep "m=" $O/qr_time_3launch.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp -o run -- python3 tools/qr_time.py 8192 > $O/rp.log 2>&1; echo "rocprof rc=$?"
python3 tools/rocpd_stats.py $O/rp/run_results.db --csv $O/qr_stats.csv > /dev/null && head -12 $O/qr_stats.csv | cut -c1-60,150-
