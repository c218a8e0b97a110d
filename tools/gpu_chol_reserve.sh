#!/bin/bash
# Cholesky lookahead: C2 stream CU reservation / priority A/B (probe_chol factor times), then C2 bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/chol_res
for R in 0 8 16 32 64; do
  SCS_CHOL_RESERVE=$R timeout -k 10 120 ./build/probe_chol > gpurun_out/chol_res/probe_r$R.log 2>&1 || { echo "probe R=$R failed"; tail gpurun_out/chol_res/probe_r$R.log; exit 1; }
  echo "R=$R $(grep factor gpurun_out/chol_res/probe_r$R.log | tr '\n' ' ')"
done
SCS_CHOL_PRIO=1 timeout -k 10 120 ./build/probe_chol > gpurun_out/chol_res/probe_prio.log 2>&1 || exit 1
echo "PRIO $(grep factor gpurun_out/chol_res/probe_prio.log | tr '\n' ' ')"
SCS_CHOL_LA=0 timeout -k 10 120 ./build/probe_chol > gpurun_out/chol_res/probe_serial.log 2>&1 || exit 1
echo "SERIAL $(grep factor gpurun_out/chol_res/probe_serial.log | tr '\n' ' ')"
for R in 0 16; do
  SCS_CHOL_RESERVE=$R timeout -k 10 240 python3 bench.py --config c2 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/chol_res/c2_r$R.json 2> gpurun_out/chol_res/c2_r$R.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/chol_res/c2_r$R.json').read().strip().splitlines()[-1]); print('c2 R=$R', d['value'], d['breakdown_ms_per_step'])"
done
