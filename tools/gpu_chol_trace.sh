#!/bin/bash
# (the probes are built here with `make -C selfconcordantsmoothoptimization.jl_amd/csrc probe` and copied to
# tools/probes/bin/probe_chol_new -- build/ does not travel to the GPU box; tools/probes/bin/ does)
# kernel trace of the Cholesky probe (factor/solve timelines at m = 8192 / 16384), summarised by
# tools/trace_chol_factor.py; then rocprofv3 --stats of the C2 bench (default configuration)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/chol_trace; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o run -- ./tools/probes/bin/probe_chol_new > $O/probe.log 2>&1 || { tail $O/probe.log; exit 1; }
python3 tools/trace_chol_factor.py $O/rp/run_kernel_trace.csv > $O/trace_summary.txt && cat $O/trace_summary.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c2 -o run -- python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline > $O/c2_bench.log 2>&1; rc=$?
echo "c2 rocprof rc=$rc"; tail -c 600 $O/c2_bench.log; find $O/c2 -name "*stats*" | head
exit $rc
