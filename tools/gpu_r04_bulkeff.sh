#!/bin/bash
# Kernel trace of the m = 65536 and m = 32768 factors (probe_chol, PROBE_SIZES) and the per-launch
# efficiency of the bulk trailing updates (tools/trace_bulk_eff.py).  Usage: gpu_r04_bulkeff.sh [outdir]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/bulkeff}; mkdir -p $O
for m in 65536 32768; do
  PROBE_SIZES=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rp$m -o run -- ./tools/probes/bin/probe_chol_sz > $O/probe$m.log 2>&1 || { tail $O/probe$m.log; exit 1; }
  python3 tools/trace_bulk_eff.py $O/rp$m/run_kernel_trace.csv $m > $O/bulk_eff_m$m.txt && cat $O/bulk_eff_m$m.txt
  rm -rf $O/rp$m
done
