#!/bin/bash
# diagonal kernel with the block load in flight: bit-identity tests, probe timings, C2 A/B vs _ab_old
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/diagload
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "cholesky or blocked or indefinite" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 ./tools/probes/bin/probe_chol_prof > $O/prof.log 2>&1 || { echo "prof failed"; tail -3 $O/prof.log; exit 1; }
grep -E "diag kernel|load |factor:" $O/prof.log
run() { # dir label
  (cd $1 && timeout -k 10 300 python3 bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-check > /tmp/dl.log 2>&1) || exit 1
  tail -1 /tmp/dl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', round(d['value'],4), {k: round(v,2) for k,v in d['breakdown_ms_per_step'].items()})"
}
for rep in 1 2; do run _ab_old old; run . new; done
