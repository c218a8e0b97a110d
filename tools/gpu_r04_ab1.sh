#!/bin/bash
# r04 A/B: the diagonal kernel's W by block columns vs the recursive doubling (probe), and the
# sparse Gram's row-block width (2^12 vs 2^11) on the C5-shaped ProxGGNSCORE step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/ab1; mkdir -p $O
for v in old new old new; do
  timeout -k 10 120 ./tools/probes/bin/probe_chol_$v >> $O/probe_$v.log 2>&1 || { echo "probe $v failed"; tail $O/probe_$v.log; exit 1; }
done
grep -H "diag kernel\|factor\|solve" $O/probe_*.log
for sh in 12 11; do
  SCS_SPARSE_GRAM_SHIFT=$sh timeout -k 10 400 python3 -u bench.py --config c5ggn --steps 2 --warmup 1 --no-cpu-baseline \
     > $O/c5ggn_shift$sh.json 2> $O/c5ggn_shift$sh.err || { echo "c5ggn $sh failed"; tail $O/c5ggn_shift$sh.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/c5ggn_shift$sh.json').read().strip().splitlines()[-1]); r=d['roofline']; print('shift $sh', d['value'], r['avg_ms'], r.get('frac'), d.get('breakdown_ms_per_step'))"
done
