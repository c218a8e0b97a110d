#!/bin/bash
# r06: the cooperative QR panel -- its parity / fallback tests, then the reference-solver QR wall time
# (tools/qr_time.py) with the per-column launches (SCS_QR_COOP=0) and the cooperative panels, alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r06/qr_coop}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "householder or reference_solver or qr_coop or qr_backward" > $O/pytest_qr.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error" $O/pytest_qr.log | tail -5; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for arm in steps coop; do
    if [ $arm = steps ]; then E="SCS_QR_COOP=0"; else E="SCS_QR_COOP=1"; fi
    env $E timeout -k 10 300 python3 -u tools/qr_time.py 2048 8192 16384 > $O/qr_${arm}_r$r.log 2>&1 || { echo "$arm failed"; tail -5 $O/qr_${arm}_r$r.log; exit 1; }
    echo "== $arm r$r"; grep "mode=2" $O/qr_${arm}_r$r.log
  done
done
