#!/bin/bash
# r06: probe_qr (tools/probes) -- the reference-solver QR solve alone: the cooperative panel with its
# per-column phase profile (-DQR_PROF), the per-column launches (default), the cooperative panel at 512 / 1024 threads
set -o pipefail
mkdir -p gpurun_out/r06/qrprof && cd gpurun_out/r06/qrprof && export PROBE_SIZES=2048,8192,16384
P=$GRAFT_REPO_ROOT/tools/probes/bin
SCS_QR_COOP=1 timeout -k 10 120 $P/probe_qr_prof > prof.log 2>&1 && SCS_QR_COOP=0 timeout -k 10 120 $P/probe_qr > steps.log 2>&1 && SCS_QR_COOP=1 timeout -k 10 120 $P/probe_qr > coop.log 2>&1 && SCS_QR_COOP=1 SCS_QR_COOP_NT=1024 timeout -k 10 120 $P/probe_qr > coop1024.log 2>&1
rc=$?; for f in prof steps coop coop1024; do echo "== $f"; cat $f.log; done; exit $rc
