#!/bin/bash
# r06 (late): the grouped QR column step's chunk rows (SCS_QR_RC) x columns per workgroup (SCS_QR_CPW),
# probe_qr alternated; then the Householder tests at the best-looking setting
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PROBE_SIZES=2048,8192,16384
tools/gpu_ab.sh gpurun_out/r06/qr_rc 2 "$GRAFT_REPO_ROOT/tools/probes/bin/probe_qr" 'n=16384' c2r1024='SCS_QR_CPW=2 SCS_QR_RC=1024' c2r512='SCS_QR_CPW=2 SCS_QR_RC=512' c2r256='SCS_QR_CPW=2 SCS_QR_RC=256' c4r512='SCS_QR_CPW=4 SCS_QR_RC=512' c4r256='SCS_QR_CPW=4 SCS_QR_RC=256' || exit 1
for f in gpurun_out/r06/qr_rc/*.log; do echo "$f $(grep n=8192 $f | tail -1 | cut -c1-32) $(grep n=2048 $f | tail -1 | cut -c1-32)"; done
