#!/bin/bash
# HEAD check: GPU suite, smoke(), default bench (C3) and the C2 line (PMC traffic attached)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/chk2
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { echo bench failed; tail -20 $O/bench_c3.err; exit 1; }
tail -1 $O/bench_c3.json | cut -c1-200
timeout -k 10 400 python bench.py --config c2 > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench c2 failed; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1]); print('c2', d['value'], d['roofline'])"
