#!/bin/bash
# r06: the block-deferred cooperative LU panel (SCS_LU_COOP_BLK=1) against the default panel: its bit
# tests, then factor + solve times alternated on one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/lu_blk; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_lu.py -k "block_deferred or variants_bit or largest_grid" > $O/t_lu.log 2>&1; rc=$?
tail -3 $O/t_lu.log; [ $rc -eq 0 ] || exit $rc
tools/gpu_ab.sh $O/time 2 'python3 tools/lu_time.py 8192 16384' 'factor_plus' blk='SCS_LU_COOP_BLK=1' base='SCS_LU_COOP_BLK=0' || exit 1
for f in $O/time/*.log; do echo $f; grep factor_plus $f; done
