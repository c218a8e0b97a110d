#!/bin/bash
# r06 (late): the QR column step with CPW panel columns per workgroup (SCS_QR_CPW) -- its bit tests, then
# probe_qr alternated over CPW = 1 / 2 / 4 / 8
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/qr_cpw; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "column_groups" > $O/t_qr.log 2>&1; rc=$?
tail -3 $O/t_qr.log; [ $rc -eq 0 ] || exit $rc
export PROBE_SIZES=2048,8192,16384
tools/gpu_ab.sh $O/time 2 "$GRAFT_REPO_ROOT/tools/probes/bin/probe_qr" 'n=16384' c1='SCS_QR_CPW=1' c2='SCS_QR_CPW=2' c4='SCS_QR_CPW=4' c8='SCS_QR_CPW=8' || exit 1
for f in $O/time/*.log; do echo $f; grep -E "n=(2048|8192)" $f | tail -2; done
