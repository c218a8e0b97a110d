#!/bin/bash
# GPU tests, then C3 / C2 bench lines with the Gram-fused Aᵀv (default) and without (SCS_GRAM_FUSE=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/fuse
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q ${PYTEST_K:+-k "$PYTEST_K"} --timeout 300 --timeout-method thread > gpurun_out/fuse/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/fuse/pytest.log; exit 1; }
tail -3 gpurun_out/fuse/pytest.log
for cfg in c3 c2; do
  timeout -k 10 240 python3 bench.py --config $cfg --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/fuse/${cfg}_fused.json 2> gpurun_out/fuse/${cfg}_fused.err || exit 1
  SCS_GRAM_FUSE=0 timeout -k 10 240 python3 bench.py --config $cfg --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/fuse/${cfg}_sep.json 2> gpurun_out/fuse/${cfg}_sep.err || exit 1
done
echo done
