#!/bin/bash
# Round-end refresh: GPU suite, smoke(), every single-GPU bench config, the C3 line + rocprofv3 stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/final
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > $O/bench_$tag.json 2> $O/bench_$tag.err || { echo "$tag failed"; tail -5 $O/bench_$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d.get('roofline',{}).get('frac'), (d.get('cpu_baseline') or {}).get('value'))"
}
run c3 --config c3
run c1 --config c1
run c2 --config c2
run c5 --config c5
run c5f32 --config c5 --f32
run c4half --config c4 --N 524288 --steps 3 --warmup 1
run c4half_cache --config c4 --N 524288 --steps 5 --warmup 1 --gram-cache
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_c3.log 2>&1 || { echo "rocprof failed"; tail $O/prof_c3.log; exit 1; }
echo done
