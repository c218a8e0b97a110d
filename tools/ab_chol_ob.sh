#!/bin/bash
# probe_chol factor times at outer block sizes SCS_CHOL_OB = 4 / 8 / 16 (8 is the default)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/ob; mkdir -p $O
for rep in 1 2; do for ob in 8 4 16 12; do
  SCS_CHOL_OB=$ob timeout -k 5 120 tools/probes/bin/probe_chol_new > $O/ob${ob}_$rep.log 2>&1 || exit 1
  echo "OB $ob rep $rep: $(grep 'factor:' $O/ob${ob}_$rep.log | awk '{print $3}' | tr '\n' ' ') $(grep 'max|x' $O/ob${ob}_$rep.log | awk '{print $NF}' | sort -g | tail -1)"
done; done
