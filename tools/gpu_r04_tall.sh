#!/bin/bash
# The bulk trailing update C12b on 256 x 128 tiles (SCS_CHOL_TALL=1) against 128 x 128 (0), at
# m = 16384 / 32768 / 65536, interleaved, twice; the U / W bit checksums must agree.
# (Run once with probe_chol built from the tall variant, tools/probes/bin/probe_chol_tall; the variant
# was bitwise equal but slower and was not kept -- profiles/r04/tall/.)
# Usage: gpu_r04_tall.sh [outdir]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/tall}; mkdir -p $O
for r in 1 2; do
  for v in 0 1; do
    SCS_CHOL_TALL=$v PROBE_SIZES=16384,32768,65536 timeout -k 10 240 ./tools/probes/bin/probe_chol_tall > $O/tall${v}_r$r.log 2>&1 \
      || { tail $O/tall${v}_r$r.log; exit 1; }
    echo "== SCS_CHOL_TALL=$v run $r"; grep -v "diag kernel" $O/tall${v}_r$r.log
  done
done
