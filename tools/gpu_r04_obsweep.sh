#!/bin/bash
# outer block size x skip threshold at m = 8192 (and 16384) with the C12 split: the factor probe, two rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/obsweep}; mkdir -p $O
for r in 1 2; do
  for ob in 3 4 5 6; do
    for t in none 800; do
      if [ $t = none ]; then env_t="SCS_CHOL_OB=$ob"; else env_t="SCS_CHOL_OB=$ob SCS_CHOL_SKIP_MAXTILES=$t"; fi
      env $env_t timeout -k 10 120 ./tools/probes/bin/probe_chol_skip > $O/ob${ob}_t${t}_r$r.log 2>&1 || { echo "ob=$ob t=$t failed"; exit 1; }
      echo "ob=$ob t=$t r=$r: $(grep 'n=8192 factor' $O/ob${ob}_t${t}_r$r.log | tail -1) | $(grep 'n=16384 factor' $O/ob${ob}_t${t}_r$r.log | tail -1)"
    done
  done
done
