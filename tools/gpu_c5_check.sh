#!/bin/bash
# C5 bench lines (fp64, fp32 values) with the full-size f / ∇f check against host SciPy
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/c5check
mkdir -p $O
for arm in f64 f32; do
  a=""; [ $arm = f32 ] && a="--f32"
  timeout -k 10 500 python3 bench.py --config c5 $a > $O/bench_$arm.json 2> $O/bench_$arm.err || { echo "bench $arm failed"; tail -5 $O/bench_$arm.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$arm.json').read().strip().splitlines()[-1]); print('$arm', round(d['value'],1), round(d['roofline']['frac'],3), d.get('parity_check'))"
done
