#!/bin/bash
# The bulk trailing update C12b in 8 x 8 super-block tile order (SCS_CHOL_SBL=1) against row-major
# (0) at m = 8192 .. 65536, interleaved, twice; U / W bit checksums must agree.
# Usage: gpu_r04_sbl.sh [outdir]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/sbl}; mkdir -p $O
for r in 1 2; do
  for v in 0 1; do
    SCS_CHOL_SBL=$v PROBE_SIZES=8192,16384,32768,65536 timeout -k 10 240 ./tools/probes/bin/probe_chol_sbl > $O/sbl${v}_r$r.log 2>&1 \
      || { tail $O/sbl${v}_r$r.log; exit 1; }
    echo "== SCS_CHOL_SBL=$v run $r"; grep "factor\|bits" $O/sbl${v}_r$r.log
  done
done
