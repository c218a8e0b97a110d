#!/bin/bash
# r06 batch 2: the cooperative-launch API against the plain launch for the LU panel (n = 8192 / 16384),
# then the whole GPU suite with durations
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/b2; mkdir -p $O
tools/gpu_ab.sh $O/lu 2 'python3 tools/lu_time.py 8192 16384' 'factor_plus' coop='SCS_LU_COOP_LAUNCH=1' plain='SCS_LU_COOP_LAUNCH=0' || exit 1
grep -h "factor_plus" $O/lu/*.log
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --timeout 600 --timeout-method thread --durations=40 tests > $O/pytest_gpu.log 2>&1; rc=$?
tail -50 $O/pytest_gpu.log
exit $rc
