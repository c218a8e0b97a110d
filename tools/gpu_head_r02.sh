#!/bin/bash
# r02 HEAD check: GPU suite, smoke(), C3 / C5 / C2 / C1 bench lines.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/head
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > $O/bench_$tag.json 2> $O/bench_$tag.err || { echo "$tag failed"; tail -5 $O/bench_$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d.get('roofline',{}).get('frac'), (d.get('cpu_baseline') or {}).get('value'))"
}
for c in ${CONFIGS:-c3 c5 c2 c1}; do run $c --config $c; done
echo done
