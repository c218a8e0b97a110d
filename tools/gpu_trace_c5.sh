#!/bin/bash
# kernel trace of a short C5 run (fp64): per-epoch kernel timeline for the gap analysis
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/c5trace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c5trace/rp -o run -- python3 bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline --no-check ${EXTRA} > gpurun_out/c5trace/bench.log 2>&1
rc=$?
# (the trace CSV is written before rocprofv3's exit: read it even after a crash at exit, but
# report the failure so the caller starts no further GPU work)
f=$(find gpurun_out/c5trace/rp -name '*kernel_trace.csv' | head -1)
[ -n "$f" ] && python3 tools/trace_gaps.py "$f" > gpurun_out/c5trace/gaps.txt && tail -40 gpurun_out/c5trace/gaps.txt
exit $rc
