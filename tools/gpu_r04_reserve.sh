#!/bin/bash
# Bulk launches sized to leave k workgroup slots free (SCS_CHOL_BULK_RESERVE=k: CU-bounded persistent
# launches of 2 ncu - k workgroups where none were bounded) vs plain launches, m = 16384 / 32768,
# interleaved, twice; U / W checksums.  Usage: gpu_r04_reserve.sh [outdir]
# (Run once with probe_chol_rsv, a build with SCS_CHOL_BULK_RESERVE; slower, not kept --
# profiles/r04/reserve/.)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/reserve}; mkdir -p $O
for r in 1 2; do
  for k in 0 2 4 16; do
    e="X=0"; [ $k -gt 0 ] && e="SCS_CHOL_BULK_RESERVE=$k"
    env $e PROBE_SIZES=16384,32768 timeout -k 10 240 ./tools/probes/bin/probe_chol_rsv > $O/k${k}_r$r.log 2>&1 \
      || { tail $O/k${k}_r$r.log; exit 1; }
    echo "== reserve $k run $r"; grep "factor\|bits" $O/k${k}_r$r.log
  done
done
