#!/bin/bash
# C2 A/B: the fused Aᵀv on 128 x 128 tiles (SCS_GRAM_FUSE=2) and 256 x 128 tiles at m = 8192
# (SCS_GRAM_TALL=1, which fuses by default) against the default (separate Aᵀv pass), two runs each,
# interleaved.  Usage: gpu_r04_c2fuse.sh [outdir]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/c2fuse}; mkdir -p $O
run() { # label env...
  local l=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline > $O/$l.json 2> $O/$l.err \
    || { echo "$l failed"; tail -3 $O/$l.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$l.json').read().strip().splitlines()[-1]); print('$l', round(d['value'],4), d.get('breakdown_ms_per_step'), (d.get('roofline') or {}).get('kernel'))"
}
for r in 1 2; do
  run def_r$r SCS_GRAM_FUSE=1 && run fuse2_r$r SCS_GRAM_FUSE=2 && run tall_r$r SCS_GRAM_TALL=1 || exit 1
done
