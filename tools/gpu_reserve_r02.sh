#!/bin/bash
# CU reserve for the Cholesky chain with the r02 diagonal kernel: solve sweep (C2, C3 shape), then
# whether rocprofv3 still crashes at exit with a CU-masked stream now that bench.py releases its
# context explicitly (last: a crash ends the call)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/rsv
for r in 0 32 48 64; do
  for c in c2 c3; do
    extra=""; [ $c = c3 ] && extra="--N 131072"
    SCS_CHOL_RESERVE_CUS=$r timeout -k 10 300 python3 bench.py --config $c $extra --steps 3 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/rsv/${c}_r$r.log 2>&1 || { echo "bench failed"; tail -3 gpurun_out/rsv/${c}_r$r.log; exit 1; }
    tail -1 gpurun_out/rsv/${c}_r$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('${c}_r$r', round(d['value'],4), round(d['breakdown_ms_per_step']['solve'],2))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rsv/rp -o run -- python3 bench.py --config c2 --steps 1 --warmup 0 --no-cpu-baseline --no-check > gpurun_out/rsv/prof.log 2>&1
echo "rocprofv3 with the default (masked) bulk stream: exit $?"
