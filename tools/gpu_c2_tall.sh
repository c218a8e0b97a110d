#!/bin/bash
# C2 Gram: 128 x 128 tiles (default at m = 8192) vs 256 x 128 tall tiles (SCS_GRAM_TALL=1), twice
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/c2tall
mkdir -p $O
for rep in 1 2; do
  for t in default 1; do
    env $( [ $t = 1 ] && echo SCS_GRAM_TALL=1 || echo X=1 ) timeout -k 10 300 python3 bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-check > $O/c2_$t.json 2> $O/c2_$t.err || { echo "bench failed"; tail -3 $O/c2_$t.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c2_$t.json').read().strip().splitlines()[-1]); print('tall=$t', round(d['value'],4), d['breakdown_ms_per_step'])"
  done
done
