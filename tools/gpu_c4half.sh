#!/bin/bash
# C4 at N = 2^19 on one GPU: the recompute line and the cached-Gram line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/c4half
mkdir -p $O
timeout -k 10 600 python3 bench.py --config c4 --N 524288 --steps 2 --warmup 1 > $O/bench_c4half.json 2> $O/bench_c4half.err || { echo "c4 failed"; tail -3 $O/bench_c4half.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c4half.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c4half', round(d['value'],4), round(r['frac'],3), r['avg_ms'], d.get('parity_check',{}).get('pass'), (d.get('cpu_baseline') or {}).get('value'))"
timeout -k 10 600 python3 bench.py --config c4 --N 524288 --gram-cache --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c4half_cache.json 2> $O/bench_c4half_cache.err || { echo "c4 cache failed"; tail -3 $O/bench_c4half_cache.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c4half_cache.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c4half cached', round(d['value'],4), round(r['frac'],3), r['avg_ms'])"
