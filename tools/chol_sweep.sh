#!/bin/bash
# Solve time (bench breakdown) against SCS_CHOL_RESERVE_CUS: m = 8192 (C2), m = 16384 (C3 shape at
# N = 2^17; the solve does not depend on N), half-size C4 with the cached Gram (m = 32768)
set -o pipefail
mkdir -p gpurun_out
for r in ${RESERVES:-0 8 16 32}; do
  SCS_CHOL_RESERVE_CUS=$r timeout -k 10 300 python3 bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline \
    --no-check > gpurun_out/c2_r$r.log 2>&1 || exit 1
  SCS_CHOL_RESERVE_CUS=$r timeout -k 10 300 python3 bench.py --config c3 --N 131072 --steps 3 --warmup 1 \
    --no-cpu-baseline --no-check > gpurun_out/c3_r$r.log 2>&1 || exit 1
  SCS_CHOL_RESERVE_CUS=$r timeout -k 10 300 python3 bench.py --config c4 --N 524288 --gram-cache --steps 2 --warmup 1 \
    --no-cpu-baseline --no-check > gpurun_out/c4_r$r.log 2>&1 || exit 1
  for f in c2_r$r c3_r$r c4_r$r; do
    tail -1 gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value'],4), round(d['breakdown_ms_per_step']['solve'],2))"
  done
done
