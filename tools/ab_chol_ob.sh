#!/bin/bash
# probe_chol factor times over outer block sizes (SCS_CHOL_OB) and bulk skip sets (SCS_CHOL_BULK_SKIP)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/ob3; mkdir -p $O
for rep in 1 2; do for cfg in "def def" "5 def" "3 def" "def 0" "def 0x30" "6 def" "10 def"; do
  set -- $cfg
  e=""; [ "$1" != def ] && e="SCS_CHOL_OB=$1"; [ "$2" != def ] && e="$e SCS_CHOL_BULK_SKIP=$2"
  env $e timeout -k 5 120 tools/probes/bin/probe_chol_new > $O/ob$1_$2_$rep.log 2>&1 || exit 1
  echo "OB $1 skip $2 rep $rep: $(grep 'factor:' $O/ob$1_$2_$rep.log | awk '{print $3}' | tr '\n' ' ') $(grep 'max|x' $O/ob$1_$2_$rep.log | awk '{print $NF}' | sort -g | tail -1)"
done; done
