#!/bin/bash
# C5 A/B: the SpMV's stream loads default vs nontemporal (SCS_SPMV_NT=1, a variant measured 10 % slower
# and not kept: profiles/r04/spmvnt/), fp64 and fp32-stored,
# interleaved, two runs each.  Usage: gpu_r04_spmvnt.sh [outdir]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/spmvnt}; mkdir -p $O
run() { # label env args...
  local l=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline "$@" > $O/$l.json 2> $O/$l.err \
    || { echo "$l failed"; tail -3 $O/$l.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$l.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$l', round(d['value'],2), r.get('kernel'), r.get('avg_ms'), round(r.get('achieved',0),1), d.get('breakdown_ms_per_step'))"
}
for r in 1 2; do
  run def_r$r SCS_SPMV_NT=0 && run nt_r$r SCS_SPMV_NT=1 && run f32def_r$r SCS_SPMV_NT=0 --f32 && run f32nt_r$r SCS_SPMV_NT=1 --f32 || exit 1
done
