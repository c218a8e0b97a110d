#!/bin/bash
# Cholesky lookahead: parity tests, then C2 / C3 bench lines with and without it (SCS_CHOL_LA=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/chol_la
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "lookahead or cache or trajectory or lu or nscore" > gpurun_out/chol_la/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/chol_la/pytest.log; exit 1; }
tail -2 gpurun_out/chol_la/pytest.log
for cfg in c2 c3; do
  timeout -k 10 240 python3 bench.py --config $cfg --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/chol_la/${cfg}_la.json 2> gpurun_out/chol_la/${cfg}_la.err || exit 1
  SCS_CHOL_LA=0 timeout -k 10 240 python3 bench.py --config $cfg --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/chol_la/${cfg}_serial.json 2> gpurun_out/chol_la/${cfg}_serial.err || exit 1
done
echo done
