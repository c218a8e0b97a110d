#!/bin/bash
# r03: CU-bounded persistent bulk launches (SCS_CHOL_BULK_SKIP) -- bit identity, then C2 A/B on one
# box against the default and the CU-masked stream, then rocprofv3 kernel stats of the best skip set.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_parity.py::test_cholesky_bounded_bulk_bit_identical" "tests/test_gpu_parity.py::test_cholesky_lookahead_bit_identical" \
  > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest.log | tail -2; [ $rc -eq 0 ] || exit $rc
b() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --config c2 --steps 6 --warmup 1 --no-cpu-baseline --no-check > $O/$n.log 2>&1 \
    || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['value'],4), 'solve_ms', round(d['breakdown_ms_per_step']['solve'],3), 'gram_ms', round(d['breakdown_ms_per_step']['gram'],2))"
}
b default
b skip20 SCS_CHOL_BULK_SKIP=0x20
b skip30 SCS_CHOL_BULK_SKIP=0x30
b skip1 SCS_CHOL_BULK_SKIP=0x1
b reserve32 SCS_CHOL_RESERVE_CUS=32
b skip20_again SCS_CHOL_BULK_SKIP=0x20
b default_again
SCS_CHOL_BULK_SKIP=0x20 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_skip20 -o run -- python3 bench.py --config c2 \
  --steps 3 --warmup 1 --no-cpu-baseline --no-check > $O/rp_skip20.log 2>&1; echo "rocprof skip20 rc=$?"
python3 tools/rocpd_stats.py $O/rp_skip20/run_results.db --csv $O/skip20_stats.csv > /dev/null && grep -E "chol_diag|gram_small|true, false, true|false, true>" $O/skip20_stats.csv | cut -c1-60,150-
