#!/bin/bash
# Cholesky factor time vs the small-Gram tile threshold (SCS_GRAM_SMALL)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/chol_small
for v in 1024 0 32 64 128 200; do
  SCS_GRAM_SMALL=$v timeout -k 10 120 ./build/probe_chol > gpurun_out/chol_small/probe_$v.log 2>&1 || { echo "probe $v failed"; tail gpurun_out/chol_small/probe_$v.log; exit 1; }
  echo "SMALL=$v $(grep -E 'factor|solve' gpurun_out/chol_small/probe_$v.log | tr '\n' ' ')"
done
