#!/bin/bash
# r03: C5 fp32-vs-fp64 tolerance study at full size, then the default-config profile run that used to
# fault at exit (CU-masked bulk stream now off by default): rocprofv3 kernel-trace stats of c2 and c3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 900 python3 -u tools/c5_tolerance.py --out $O/tolerance.json > $O/tol.log 2>&1
rc=$?; echo "tolerance rc=$rc"; tail -3 $O/tol.log; [ $rc -eq 0 ] || exit $rc
SCS_SEGV_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_c2 -o run -- python3 bench.py --config c2 \
  --steps 3 --warmup 1 --no-cpu-baseline --no-check > $O/prof_c2.log 2>&1
rc=$?; echo "rocprofv3 default c2: exit $rc"; tail -c 600 $O/prof_c2.log; [ $rc -eq 0 ] || exit $rc
