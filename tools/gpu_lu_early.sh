#!/bin/bash
# r06: the record-first cooperative LU panel (SCS_LU_COOP_EARLY, default 1) against r05's order (=0):
# the LU tests (pivots / bits against the column steps and LAPACK), per-column phases, factor + solve times
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/lu_early; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lu.py tests/test_gpu_fallback.py > $O/t_lu.log 2>&1; rc=$?
tail -3 $O/t_lu.log; [ $rc -eq 0 ] || exit $rc
for a in 1 0; do SCS_LU_COOP_EARLY=$a PROBE_SIZES=8192,16384 timeout -k 10 300 ./tools/probes/bin/probe_lu_prof > $O/prof_early$a.log 2>&1 || exit 1; echo "early=$a"; cat $O/prof_early$a.log; done
tools/gpu_ab.sh $O/time 2 'python3 tools/lu_time.py 8192 16384' 'factor_plus' early='SCS_LU_COOP_EARLY=1' r05='SCS_LU_COOP_EARLY=0' || exit 1
for f in $O/time/*.log; do echo $f; grep factor_plus $f; done
