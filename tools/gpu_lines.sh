#!/bin/bash
# One bench line per configuration on the current build (default configuration, no env overrides):
# c2, c4 at N = 2^19 with the cached Gram (c4 needs >= 4 GPUs at full size), c5 fp64 / fp32-stored, c5ggn, c1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/lines}; mkdir -p $O
line() { # label args...
  local l=$1; shift
  timeout -k 10 500 python3 bench.py "$@" > $O/$l.json 2> $O/$l.err || { echo "$l failed"; tail -3 $O/$l.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$l.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$l', round(d['value'],4), d['unit'], r.get('kernel'), round(r.get('frac',0),4), d.get('breakdown_ms_per_step'), (d.get('cpu_baseline') or {}).get('value'))"
}
line c2 --config c2 --steps 10 --warmup 2 && line c4half_cache --config c4 --N 524288 --gram-cache --steps 5 --warmup 1 && line c5 --config c5 && line c5_f32 --config c5 --f32 && line c5ggn --config c5ggn --steps 2 --warmup 1 --no-cpu-baseline && line c1 --config c1
