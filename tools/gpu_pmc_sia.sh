#!/bin/bash
# L2 hit/miss of the interleaved Gram kernel vs rocBLAS DGEMM at K = 65536, m = 16384
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_sia
for v in 9 11; do
  GRAM_ONLY=$v timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_sia/k$v -o run -- ./build/probe_gram 65536 16384 1 > gpurun_out/pmc_sia/k$v.log 2>&1 || { echo "pmc k$v failed"; exit 1; }
done
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_sia/rb -o run -- python3 tools/probe_rocblas_k64.py > gpurun_out/pmc_sia/rb.log 2>&1 || { echo "pmc rocblas failed"; exit 1; }
find gpurun_out/pmc_sia -name "*counter_collection.csv" | head
