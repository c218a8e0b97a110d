#!/bin/bash
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o run -- python3 bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc
