#!/bin/bash
# A/B of SCS_CHOL_SKIP_MAXTILES (bulk launches above the threshold use every CU): the factor probe
# (m = 8192 / 16384), one process per setting, two rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/skip}; mkdir -p $O
for r in 1 2; do
  for t in none 3000 1500 800 400; do
    if [ $t = none ]; then env_t=""; else env_t="SCS_CHOL_SKIP_MAXTILES=$t"; fi
    env $env_t timeout -k 10 120 ./tools/probes/bin/probe_chol_skip > $O/t${t}_r$r.log 2>&1 || { echo "t=$t failed"; exit 1; }
    echo "t=$t r=$r: $(grep 'n=8192 factor' $O/t${t}_r$r.log | tail -1) | $(grep 'n=16384 factor' $O/t${t}_r$r.log | tail -1)"
  done
done
