#!/bin/bash
# r06 batch 1: the fallback tests, the LU / Cholesky suites on the new build, then the packed diagonal
# kernel A/B (tools/gpu_chol_pack.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/b1; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=15 \
  tests/test_gpu_fallback.py tests/test_gpu_lu.py > $O/t_fallback_lu.log 2>&1; rc=$?
tail -5 $O/t_fallback_lu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=15 \
  tests/test_gpu_parity.py -k "cholesky or solve or pipelined or lookahead" > $O/t_chol.log 2>&1; rc=$?
tail -5 $O/t_chol.log
[ $rc -eq 0 ] || exit $rc
tools/gpu_chol_pack.sh
