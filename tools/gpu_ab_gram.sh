#!/bin/bash
# same-box A/B of the default Gram path: this tree vs _ab_old (C3 at N/4 and C2, twice)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
run() { # dir label args
  (cd $1 && timeout -k 10 300 python3 bench.py $3 --steps 3 --warmup 1 --no-cpu-baseline --no-check > /tmp/abg.log 2>&1) || exit 1
  tail -1 /tmp/abg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', round(d['value'],4), {k: round(v,2) for k,v in d['breakdown_ms_per_step'].items()})"
}
for rep in 1 2; do
  run _ab_old old-c3q "--config c3 --N 262144"
  run . new-c3q "--config c3 --N 262144"
  run _ab_old old-c2 "--config c2"
  run . new-c2 "--config c2"
done
