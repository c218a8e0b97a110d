#!/bin/bash
# C2 / half-size C4 (cached Gram) solve time against SCS_CHOL_RESERVE_CUS (bench lines -> gpurun_out/)
set -o pipefail
mkdir -p gpurun_out
for r in ${RESERVES:-0 16 32}; do
  SCS_CHOL_RESERVE_CUS=$r timeout -k 10 300 python3 bench.py --config c4 --N 524288 --gram-cache --steps 2 --warmup 1 \
    --no-cpu-baseline --no-check > gpurun_out/c4_r$r.log 2>&1 || exit 1
  SCS_CHOL_RESERVE_CUS=$r timeout -k 10 300 python3 bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline \
    --no-check > gpurun_out/c2_r$r.log 2>&1 || exit 1
  for f in c4_r$r c2_r$r; do
    tail -1 gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value'],4), d['breakdown_ms_per_step']['solve'])"
  done
done
