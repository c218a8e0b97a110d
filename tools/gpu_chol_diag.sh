#!/bin/bash
# diagonal-kernel schedule: bit-identity tests, then the C2 solve A/B (SCS_CHOL_DIAG=0 vs default)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/cholpipe
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "cholesky or blocked or indefinite" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for d in 0 1; do
    SCS_CHOL_ILA=$d timeout -k 10 300 python3 bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-check > $O/c2_d$d.json 2> $O/c2_d$d.err || { echo "bench failed"; tail $O/c2_d$d.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c2_d$d.json').read().strip().splitlines()[-1]); print('ila=$d', round(d['value'],3), d['breakdown_ms_per_step'])"
  done
done
timeout -k 10 120 ./tools/probes/bin/probe_chol_prof > $O/prof.log 2>&1 || { echo "prof failed"; tail $O/prof.log; exit 1; }
grep -E "diag kernel|load|factor:" $O/prof.log
