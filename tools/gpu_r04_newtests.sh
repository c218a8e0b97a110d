#!/bin/bash
# the r04 additions' GPU tests (host-exchange groups, held-out golden cases) in one process
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/newtests}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_multi.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "multi or heldout" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $O/pytest.log; exit $rc
