#!/bin/bash
# one-launch Gram with per-strip counts + the factor behind it (SCS_CHOL_PIPE=2): parity tests,
# then C2 / C3 lines with the pipeline off / per-strip launches / one launch
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pipe2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "pipelined" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for p in 0 2; do
    SCS_CHOL_PIPE=$p timeout -k 10 300 python3 bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-check > $O/c2_p$p.json 2> $O/c2_p$p.err || { echo "bench failed"; tail -3 $O/c2_p$p.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c2_p$p.json').read().strip().splitlines()[-1]); print('c2 pipe=$p', round(d['value'],4), {k: round(v,2) for k,v in d['breakdown_ms_per_step'].items()})"
  done
done
for p in 0 2; do
  SCS_CHOL_PIPE=$p timeout -k 10 300 python3 bench.py --config c3 --N 262144 --steps 3 --warmup 1 --no-cpu-baseline --no-check > $O/c3q_p$p.json 2> $O/c3q_p$p.err || { echo "bench failed"; tail -3 $O/c3q_p$p.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3q_p$p.json').read().strip().splitlines()[-1]); print('c3 N/4 pipe=$p', round(d['value'],4), {k: round(v,2) for k,v in d['breakdown_ms_per_step'].items()})"
done
