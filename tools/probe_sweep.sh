#!/bin/bash
# probe_chol (factor + solve at m = 8192 / 16384) under each given environment setting, twice, one box.
# usage: probe_sweep.sh [outdir] "SCS_CHOL_OB=4" "SCS_CHOL_OB=8 SCS_CHOL_BULK_SKIP=0" "SCS_GRAM_SMALL=64" ...
# ("-" = the defaults).  The probe is built here (make -C selfconcordantsmoothoptimization.jl_amd/csrc probe)
# and copied to tools/probes/bin/probe_chol_new: build/ does not travel to the GPU box.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/sweep}; shift; mkdir -p $O
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i + 1)); e=""; [ "$cfg" != "-" ] && e="$cfg"
    env $e timeout -k 5 120 tools/probes/bin/probe_chol_new > $O/cfg${i}_$rep.log 2>&1 || { echo "failed: $cfg"; exit 1; }
    echo "[$cfg] rep $rep: factor ms $(grep 'factor:' $O/cfg${i}_$rep.log | awk '{print $3}' | tr '\n' ' ') max|x-1| $(grep 'max|x' $O/cfg${i}_$rep.log | awk '{print $NF}' | sort -g | tail -1)"
  done
done
