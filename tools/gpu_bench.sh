#!/bin/bash
# Full-size bench + rocprofv3 kernel-trace stats (used with gpurun).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python bench.py > gpurun_out/bench_full.log 2> gpurun_out/bench_full.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_full.log; tail -3 gpurun_out/bench_full.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r01 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r01.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_r01.log
find gpurun_out/prof_r01 -name "*stats*" | head
exit $rc
