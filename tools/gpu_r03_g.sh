#!/bin/bash
# r03: C2 factor chain vs the bulk stream without a CU mask -- stream priorities (SCS_CHOL_BULK_PRIO
# 1: bulk low, 2: + context stream high) against the default and the r02 CU reserve, same box; then
# kernel stats of the best priority setting; last, the CU-masked stream kept alive to process exit
# under rocprofv3 (diagnosis of the exit fault).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03g; mkdir -p $O
b() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --config c2 --steps 6 --warmup 1 --no-cpu-baseline --no-check > $O/$n.log 2>&1 \
    || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['value'],4), 'solve_ms', round(d['breakdown_ms_per_step']['solve'],3), 'gram_ms', round(d['breakdown_ms_per_step']['gram'],2))"
}
b default
b prio1 SCS_CHOL_BULK_PRIO=1
b prio2 SCS_CHOL_BULK_PRIO=2
b reserve32 SCS_CHOL_RESERVE_CUS=32
b prio2_reserve32 SCS_CHOL_BULK_PRIO=2 SCS_CHOL_RESERVE_CUS=32
b default_again
SCS_CHOL_BULK_PRIO=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_prio2 -o run -- python3 bench.py --config c2 \
  --steps 3 --warmup 1 --no-cpu-baseline --no-check > $O/rp_prio2.log 2>&1; echo "rocprof prio2 rc=$?"
python3 tools/rocpd_stats.py $O/rp_prio2/run_results.db --csv $O/prio2_stats.csv > /dev/null && grep -E "chol_diag|gram_small" $O/prio2_stats.csv | cut -c1-40,160-
SCS_CHOL_RESERVE_CUS=32 SCS_CHOL_KEEP_BULK=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_keep -o run -- python3 bench.py --config c2 \
  --steps 1 --warmup 0 --no-cpu-baseline --no-check > $O/rp_keep.log 2>&1; echo "rocprof reserve32 keep-bulk rc=$?"
tail -3 $O/rp_keep.log
