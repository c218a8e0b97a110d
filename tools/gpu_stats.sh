#!/bin/bash
# rocprofv3 --kernel-trace --stats of the default bench lines (C3, C2, C5, C5-shaped GGN) on the current build:
# per-kernel CSV summaries + the bench line measured under the profiler
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/stats}; mkdir -p $O
prof() {  # label, bench args...
  local l=$1; shift
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/$l -o run -- python3 bench.py "$@" --no-cpu-baseline \
    > $O/$l.log 2>&1 || { echo "$l failed"; tail -5 $O/$l.log; return 1; }
  python3 tools/rocpd_stats.py $O/$l/run_results.db --csv $O/${l}_kernel_stats.csv > /dev/null || return 1
  grep '"metric"' $O/$l.log | tail -1 > $O/bench_${l}_under_rocprof.json
  echo "== $l"; head -6 $O/${l}_kernel_stats.csv | cut -c1-150
  rm -rf $O/$l
}
prof c3 --steps 2 --warmup 1 && prof c2 --config c2 --steps 5 --warmup 1 && prof c5 --config c5 \
  && prof c5ggn --config c5ggn --steps 2 --warmup 1
