#!/bin/bash
# C5 bench SpMV time against SCS_SPMV_RW x SCS_SPMV_CHUNKS (fp64 and fp32 arms)
set -o pipefail
mkdir -p gpurun_out
for arm in "" "--f32"; do
  for rw in ${RWS:-2 4 8}; do
    for ch in ${CHS:-1 2 4}; do
      SCS_SPMV_RW=$rw SCS_SPMV_CHUNKS=$ch timeout -k 10 200 python3 bench.py --config c5 $arm --steps 20 --warmup 3 \
        --no-cpu-baseline --no-check > gpurun_out/sw.log 2>&1 || exit 1
      tail -1 gpurun_out/sw.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm rw=$rw ch=$ch', round(d['value'],1), round(d['roofline']['avg_ms'],4))"
    done
  done
done
