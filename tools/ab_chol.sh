#!/bin/bash
# (old = a build of the comparison commit in _ab_old/, new = this tree; probes copied to tools/probes/bin/
# as probe_chol_{old,new}[_prof] beforehand -- build/ does not travel to the GPU box)
# A/B of the Cholesky factor: the library built from HEAD in _ab_old/ against the working tree,
# probe_chol (diag kernel alone, factor, solve) and bench --config c2, alternated; then the
# factor's bit-identity tests on the new build.  Usage: ab_chol.sh [outdir]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/abchol}; mkdir -p $O
P=tools/probes/bin
for v in old new; do
  timeout -k 10 120 $P/probe_chol_$v > $O/probe_$v.log 2>&1 || { echo "probe $v failed"; tail -5 $O/probe_$v.log; exit 1; }
  echo "== $v"; head -4 $O/probe_$v.log; grep "n=16384" $O/probe_$v.log
  if [ -x $P/probe_chol_prof_$v ]; then
    timeout -k 10 120 $P/probe_chol_prof_$v > $O/probe_prof_$v.log 2>&1 || { echo "probe_prof $v failed"; exit 1; }
    sed -n 2,4p $O/probe_prof_$v.log
  fi
done
run() { # dir label
  (cd $1 && timeout -k 10 300 python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --no-check > /tmp/abc2.log 2>&1) || { tail -5 /tmp/abc2.log; exit 1; }
  cp /tmp/abc2.log $O/bench_c2_$2.json
  tail -1 /tmp/abc2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); t=d.get('breakdown_ms_per_step',{}); print('$2', round(d['value'],3), {k: round(v,2) for k,v in t.items()})"
}
for rep in 1 2; do run _ab_old old$rep; run . new$rep; done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "cholesky or chol or lu or qr or default_path or solve" > $O/pytest_chol.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest_chol.log; exit $rc
