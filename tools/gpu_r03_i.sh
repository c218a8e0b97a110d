#!/bin/bash
# r03: the CU-bounded bulk launches as the default up to m = 16384 -- factor bit-identity tests, then
# same-box A/B (default vs SCS_CHOL_BULK_SKIP=0) at C2 (m = 8192), the C3 shape at N/8 (m = 16384)
# and C4-half with the cached Gram (m = 32768, default there: no skip; 0x20 forced for comparison).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03i; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_parity.py::test_cholesky_bounded_bulk_bit_identical" "tests/test_gpu_parity.py::test_cholesky_lookahead_bit_identical" \
  "tests/test_gpu_parity.py::test_cholesky_diag_pipe_bit_identical" "tests/test_gpu_default_path.py" \
  > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest.log | tail -2; [ $rc -eq 0 ] || exit $rc
b() {  # name, args, env...
  local n=$1; local a=$2; shift 2
  env "$@" timeout -k 10 400 python3 bench.py $a --no-cpu-baseline --no-check > $O/$n.log 2>&1 \
    || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['value'],4), 'solve_ms', round(d['breakdown_ms_per_step']['solve'],3), 'gram_ms', round(d['breakdown_ms_per_step']['gram'],2))"
}
b c2_default "--config c2 --steps 6 --warmup 1"
b c2_skip0 "--config c2 --steps 6 --warmup 1" SCS_CHOL_BULK_SKIP=0
b c3n8_default "--config c3 --N 131072 --steps 4 --warmup 1"
b c3n8_skip0 "--config c3 --N 131072 --steps 4 --warmup 1" SCS_CHOL_BULK_SKIP=0
b c4h_default "--config c4 --N 524288 --steps 4 --warmup 1 --gram-cache"
b c4h_skip20 "--config c4 --N 524288 --steps 4 --warmup 1 --gram-cache" SCS_CHOL_BULK_SKIP=0x20
b c2_default_again "--config c2 --steps 6 --warmup 1"
b c3n8_default_again "--config c3 --N 131072 --steps 4 --warmup 1"
