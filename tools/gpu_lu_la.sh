#!/bin/bash
# r06: the LU's lookahead outer step (SCS_LU_LA=1) -- its bit tests, then factor + solve times against the
# one-stream step, alternated on one box, with the bulk's skip sets
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/lu_la; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_lu.py -k "lookahead" > $O/t_lu.log 2>&1; rc=$?
tail -3 $O/t_lu.log; [ $rc -eq 0 ] || exit $rc
tools/gpu_ab.sh $O/time 3 'python3 tools/lu_time.py 8192 16384' 'factor_plus' base='SCS_LU_LA=0' auto='SCS_LU_LA=1' full4k='SCS_LU_LA=1 SCS_LU_LA_FULL=4096' full12k='SCS_LU_LA=1 SCS_LU_LA_FULL=12288' la0='SCS_LU_LA=1 SCS_LU_LA_SKIP=0' || exit 1
for f in $O/time/*.log; do echo $f; grep factor_plus $f; done
