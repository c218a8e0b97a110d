#!/bin/bash
# probe_chol factor times over SCS_GRAM_SMALL (max tiles a gen launch sends to the latency kernel)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/small; mkdir -p $O
for rep in 1 2; do for v in 64 32 128 256; do
  SCS_GRAM_SMALL=$v timeout -k 5 120 tools/probes/bin/probe_chol_new > $O/s${v}_$rep.log 2>&1 || exit 1
  echo "small $v rep $rep: $(grep 'factor:' $O/s${v}_$rep.log | awk '{print $3}' | tr '\n' ' ') $(grep 'max|x' $O/s${v}_$rep.log | awk '{print $NF}' | sort -g | tail -1)"
done; done
