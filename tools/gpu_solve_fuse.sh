#!/bin/bash
# one-launch triangular-solve steps: tests (bit identity, solves, LU fallback), probe solve times, C2 A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/sfuse
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_default_path.py -m gpu -x -v --timeout 300 --timeout-method thread -k "cholesky or blocked or indefinite or c2 or C2 or c4 or C4 or nscore" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for f in 0 1; do
  SCS_SOLVE_FUSE=$f timeout -k 10 120 ./tools/probes/bin/probe_chol > $O/probe_f$f.log 2>&1 || { echo "probe failed"; tail -3 $O/probe_f$f.log; exit 1; }
  echo "fuse=$f"; grep "solve:" $O/probe_f$f.log
done
for rep in 1 2; do
  for f in 0 1; do
    SCS_SOLVE_FUSE=$f timeout -k 10 300 python3 bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-check > $O/c2_f$f.json 2> $O/c2_f$f.err || { echo "bench failed"; tail -3 $O/c2_f$f.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c2_f$f.json').read().strip().splitlines()[-1]); print('c2 fuse=$f', round(d['value'],4), {k: round(v,2) for k,v in d['breakdown_ms_per_step'].items()})"
  done
done
