#!/bin/bash
# Outer block 8 / 12 / 16 (SCS_CHOL_OB) at m = 32768 / 65536, where the bulk stream's K = OB * 128
# trailing updates bound the factor; interleaved, twice.  Usage: gpu_r04_obbig.sh [outdir]
# (probe_chol_tall: probe_chol with PROBE_SIZES, built from the r04 tall-variant tree; any probe_chol
# build with PROBE_SIZES gives the same OB sweep.)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/obbig}; mkdir -p $O
for r in 1 2; do
  for ob in 8 12 16; do
    SCS_CHOL_OB=$ob PROBE_SIZES=32768,65536 timeout -k 10 240 ./tools/probes/bin/probe_chol_tall > $O/ob${ob}_r$r.log 2>&1 \
      || { tail $O/ob${ob}_r$r.log; exit 1; }
    echo "== SCS_CHOL_OB=$ob run $r"; grep "factor\|bits" $O/ob${ob}_r$r.log
  done
done
