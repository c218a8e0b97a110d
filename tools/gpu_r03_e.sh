#!/bin/bash
# r03 A/B of the chain launches' synchronization cost at C2: polling sleep and (timing only) no
# agent-scope fences, under rocprofv3 kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03e; mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_$n -o run -- python3 bench.py --config c2 --steps 3 \
    --warmup 1 --no-cpu-baseline --no-check > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }
  python3 tools/rocpd_stats.py $O/rp_$n/run_results.db --csv $O/$n.csv > /dev/null
  grep '^{' $O/$n.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['value'],4), 'solve_ms', round(d['breakdown_ms_per_step']['solve'],3))"
  python3 -c "
import csv
for r in csv.DictReader(open('$O/$n.csv')):
    n=r['Name'].split('(')[0][-30:]
    if 'dag' in n or 'chol_diag' in n: print('   ', n, r['Calls'], r['AverageUs'])
"
}
run dag_s1 SCS_CHOL_DAG=1
run dag_s16 SCS_CHOL_DAG=1 SCS_CHOL_DAG_SLEEP=16
run dag_nofence SCS_CHOL_DAG=1 SCS_CHOL_DAG_FENCE=0
run dag_off SCS_CHOL_DAG=0
