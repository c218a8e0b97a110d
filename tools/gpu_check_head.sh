#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/chk
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/chk/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/chk/pytest.log; exit 1; }
tail -2 gpurun_out/chk/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/chk/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/chk/smoke.log; exit 1; }
tail -1 gpurun_out/chk/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/chk/bench.log 2> gpurun_out/chk/bench.err || { echo bench failed; tail -20 gpurun_out/chk/bench.err; exit 1; }
tail -1 gpurun_out/chk/bench.log | cut -c1-900
