#!/bin/bash
# Phase A of the diagonal kernel: the r03 order against the deferred LDS-fed updates
# (SCS_CHOL_PHASEA=1), interleaved, twice: diagonal kernel alone, factor + solve at m = 8192 / 16384,
# and the U / W bit checksums (must agree).  Then the CHOL_PROF build's phase times for both.
# (Run once with probe_chol built from the DFR variant, tools/probes/bin/probe_chol_pa{,_prof}; the
# variant measured no faster and was not kept -- profiles/r04/phasea/.)
# Usage: gpu_r04_phasea.sh [outdir]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/phasea}; mkdir -p $O
for r in 1 2; do
  for v in 0 1; do
    SCS_CHOL_PHASEA=$v timeout -k 10 120 ./tools/probes/bin/probe_chol_pa > $O/pa${v}_r$r.log 2>&1 || { tail $O/pa${v}_r$r.log; exit 1; }
    echo "== PHASEA=$v run $r"; cat $O/pa${v}_r$r.log
  done
done
for v in 0 1; do
  SCS_CHOL_PHASEA=$v timeout -k 10 120 ./tools/probes/bin/probe_chol_pa_prof > $O/prof${v}.log 2>&1 || { tail $O/prof${v}.log; exit 1; }
  echo "== prof PHASEA=$v"; head -4 $O/prof${v}.log
done
