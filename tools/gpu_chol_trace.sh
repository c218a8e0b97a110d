#!/bin/bash
# kernel trace of the Cholesky probe (factor/solve timelines at m = 8192 / 16384)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/chol_trace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/chol_trace/rp -o run -- ./tools/probes/bin/probe_chol > gpurun_out/chol_trace/probe.log 2>&1 || { tail gpurun_out/chol_trace/probe.log; exit 1; }
cat gpurun_out/chol_trace/probe.log | grep factor
