#!/bin/bash
# r06 (late): the two-operand K = 128 products (the QR's trailing update A -= V Y, the LU's TRSM) on the
# interleaved kernel (SCS_GRAM_SIA2=1) against gram_f64_kernel, probe_qr and the LU, alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PROBE_SIZES=8192,16384
tools/gpu_ab.sh gpurun_out/r06/sia2_k128/qr 2 "$GRAFT_REPO_ROOT/tools/probes/bin/probe_qr" 'n=16384' base='SCS_GRAM_SIA2=' sia2='SCS_GRAM_SIA2=1' || exit 1
tools/gpu_ab.sh gpurun_out/r06/sia2_k128/lu 2 'python3 tools/lu_time.py 8192 16384' 'factor_plus' base='SCS_GRAM_SIA2=' sia2='SCS_GRAM_SIA2=1' || exit 1
grep -h "n=8192" gpurun_out/r06/sia2_k128/qr/*.log | tail -4; grep -h '"n": 8192' gpurun_out/r06/sia2_k128/lu/*.log | cut -c1-80
