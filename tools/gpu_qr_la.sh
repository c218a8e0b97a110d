#!/bin/bash
# r06: the QR's lookahead trailing update (SCS_QR_LA=1) -- its bit tests and the Householder tests, then
# probe_qr (the reference-solver QR solve alone) against the one-stream update, alternated on one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/qr_la; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "qr_lookahead or householder" > $O/t_qr.log 2>&1; rc=$?
tail -3 $O/t_qr.log; [ $rc -eq 0 ] || exit $rc
export PROBE_SIZES=2048,8192,16384
tools/gpu_ab.sh $O/time 3 "$GRAFT_REPO_ROOT/tools/probes/bin/probe_qr" 'n=16384' base='SCS_QR_LA=0' la='SCS_QR_LA=1' || exit 1
for f in $O/time/*.log; do echo $f; cat $f; done
