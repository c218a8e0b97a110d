#!/bin/bash
# SpMV A/B (env switches in $@ as NAME=VAL pairs, each run separately): sparse GPU tests, C5 fp64 + fp32 bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/spmv_ab
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 120 --timeout-method thread > gpurun_out/spmv_ab/pytest_$cfg.log 2>&1 || { echo "pytest $cfg failed"; tail -30 gpurun_out/spmv_ab/pytest_$cfg.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/spmv_ab/pytest_$cfg.log)"
  for f in "" "--f32"; do
    env $cfg timeout -k 10 300 python3 bench.py --config c5 $f --no-cpu-baseline > gpurun_out/spmv_ab/c5_$cfg$f.json 2> gpurun_out/spmv_ab/c5_$cfg$f.err || { echo "bench failed"; tail gpurun_out/spmv_ab/c5_$cfg$f.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/spmv_ab/c5_$cfg$f.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c5 $cfg $f', round(d['value'],1), 'spmv avg ms', round(r['avg_ms'],4), 'GB/s', round(r['achieved']))"
  done
done
