#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PROBE_SIZES=2048,8192,16384
tools/gpu_ab.sh gpurun_out/r06/qr_la/coop 2 "$GRAFT_REPO_ROOT/tools/probes/bin/probe_qr" 'n=16384' coop='SCS_QR_COOP=1 SCS_QR_LA=0' coopla='SCS_QR_COOP=1 SCS_QR_LA=1'
