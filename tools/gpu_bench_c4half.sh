#!/bin/bash
# C4 at N = 2^19 on one GPU (recompute mode), bench line with cpu_baseline and PMC traffic
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/c4h
timeout -k 10 500 python -u bench.py --config c4 --N 524288 --steps 3 --warmup 1 > gpurun_out/c4h/bench_c4half.json 2> gpurun_out/c4h/bench_c4half.err || { tail -5 gpurun_out/c4h/bench_c4half.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/c4h/bench_c4half.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline'])"
