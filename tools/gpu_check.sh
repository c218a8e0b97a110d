#!/bin/bash
# Round-end gate rehearsal: the whole GPU suite, smoke() and the default bench line,
# each under its own time limit; stops at the first failure.  Usage: gpu_check.sh [outdir]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/check}; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc=$rc"; tail -c 1500 $O/bench.json
exit $rc
