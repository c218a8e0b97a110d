#!/bin/bash
# the C4 per-rank-shape test, then the C5-shaped GGN line with fp32-stored values (variant 8 <float>)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/c4f32}; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_full_size.py -m gpu -x -v --timeout 600 --timeout-method thread \
  -p no:cacheprovider --durations=0 -k "c4" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -6 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --config c5ggn --f32 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5ggn_f32.json \
  2> $O/c5ggn_f32.err || { tail -3 $O/c5ggn_f32.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c5ggn_f32.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c5ggn f32', round(d['value'],4), r.get('kernel'), r.get('avg_ms'), d.get('breakdown_ms_per_step'))"
