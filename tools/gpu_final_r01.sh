#!/bin/bash
# Round-end check: the GPU test suite, smoke(), then the C3 bench + rocprof stats + PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/final/pytest.log; exit 1; }
tail -2 gpurun_out/final/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -2 gpurun_out/final/smoke.log
bash tools/gpu_prof_c3.sh
