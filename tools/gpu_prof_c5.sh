#!/bin/bash
# C5 bench line + rocprofv3 kernel-trace stats of the same command (kernel list, per-step gaps)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof_c5
timeout -k 10 300 python3 bench.py --config c5 > gpurun_out/prof_c5/bench.json 2> gpurun_out/prof_c5/bench.err || { tail gpurun_out/prof_c5/bench.err; exit 1; }
tail -1 gpurun_out/prof_c5/bench.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5/rp -o run -- python3 bench.py --config c5 --no-cpu-baseline > gpurun_out/prof_c5/rp.log 2>&1 || { tail gpurun_out/prof_c5/rp.log; exit 1; }
find gpurun_out/prof_c5/rp -name "*.csv" | head
