#!/bin/bash
# Stream priorities for the factor's two streams: plain, bulk stream low (SCS_CHOL_BULK_PRIO=1),
# chain stream high (PROBE_CHAIN_PRIO=-1), both; m = 8192 / 16384 / 32768, interleaved, twice.
# (Run once with probe_chol_prio: probe_chol + PROBE_CHAIN_PRIO, and chol.hip + SCS_CHOL_BULK_PRIO;
# no measurable effect, not kept -- profiles/r04/prio/.)
# Usage: gpu_r04_prio.sh [outdir]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/prio}; mkdir -p $O
for r in 1 2; do
  i=0
  for cfg in "X=0" "SCS_CHOL_BULK_PRIO=1" "PROBE_CHAIN_PRIO=-1" "SCS_CHOL_BULK_PRIO=1 PROBE_CHAIN_PRIO=-1"; do
    i=$((i + 1))
    env $cfg PROBE_SIZES=8192,16384,32768 timeout -k 10 240 ./tools/probes/bin/probe_chol_prio > $O/cfg${i}_r$r.log 2>&1 \
      || { tail $O/cfg${i}_r$r.log; exit 1; }
    echo "== $cfg run $r"; grep "factor\|bits\|range" $O/cfg${i}_r$r.log
  done
done
