#!/bin/bash
# r06 (late): rocprofv3 kernel stats of the reference-solver QR solve alone (probe_qr, n = 8192, 3 solves)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/qrstats; mkdir -p $O
PROBE_SIZES=8192 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o qr -- "$GRAFT_REPO_ROOT/tools/probes/bin/probe_qr" > $O/run.log 2>&1; rc=$?
cat $O/run.log | grep qr_solve; find $O/prof -name "*stats*" | head; exit $rc
