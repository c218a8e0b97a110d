#!/bin/bash
# r06 (late): the block-deferred LU panel at 512-thread workgroups (256 rows each, half the records per
# sweep) against the default 256, with the lookahead outer step, alternated on one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu_ab.sh gpurun_out/r06/lu_nt 3 'python3 tools/lu_time.py 8192 16384' 'factor_plus' nt256='SCS_LU_COOP_NT=256' nt512='SCS_LU_COOP_NT=512'
