#!/bin/bash
# full-size parity tests (C2 trajectory vs the oracle, C3 sampled Gram + a step, C5 f / ∇f vs SciPy)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/full}; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_full_size.py -m gpu -x -v --timeout 900 --timeout-method thread \
  -p no:cacheprovider --durations=0 > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -12 $O/pytest.log; exit $rc
