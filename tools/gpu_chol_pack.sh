#!/bin/bash
# r06: the packed-LDS diagonal kernel (SCS_CHOL_DIAG_PACK=1, default) against r05's full copy (=0):
# factor-probe A/B (bits of U / W must agree across arms), then the probe's kernel trace summarised
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/pack; mkdir -p $O
tools/gpu_ab.sh $O 2 './tools/probes/bin/probe_chol_new' 'factor' pack='SCS_CHOL_DIAG_PACK=1' full='SCS_CHOL_DIAG_PACK=0' || exit 1
grep -h "bits\|diag kernel\|solve:" $O/*.log | sort | uniq -c
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o run -- ./tools/probes/bin/probe_chol_new > $O/probe_trace.log 2>&1 || { tail $O/probe_trace.log; exit 1; }
python3 tools/trace_chol_factor.py $O/rp/run_kernel_trace.csv > $O/chol_trace_summary.txt && cat $O/chol_trace_summary.txt
# in-kernel times of the diagonal kernels (probe_chol_dtime), both layouts
for arm in 1 0; do SCS_CHOL_DIAG_PACK=$arm timeout -k 10 300 ./tools/probes/bin/probe_chol_dtime > $O/dtime_pack$arm.log 2>&1 || exit 1; echo "pack=$arm"; grep -h "in-kernel\|factor:" $O/dtime_pack$arm.log; done
