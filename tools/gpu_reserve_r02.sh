#!/bin/bash
# CU reserve for the Cholesky chain with the r02 diagonal kernel: solve sweep, then whether rocprofv3
# still crashes at exit in a process that created a CU-masked stream (last: a crash ends the call)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
RESERVES="0 16 32" bash tools/chol_sweep.sh || { echo "sweep failed"; exit 1; }
mkdir -p gpurun_out/rsv
SCS_CHOL_RESERVE_CUS=32 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rsv/rp -o run -- python3 bench.py --config c2 --steps 1 --warmup 0 --no-cpu-baseline --no-check > gpurun_out/rsv/prof.log 2>&1
echo "rocprofv3 with a masked stream: exit $?"
