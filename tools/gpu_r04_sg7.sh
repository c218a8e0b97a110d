#!/bin/bash
# sparse Gram variants 8 (table-driven walk), 6, 7 (half-batch pipeline): bitwise test + C5-shaped GGN bench each
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/sg7}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_sparse.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "gram" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 8 6 7 8; do
  SCS_SPARSE_GRAM_KERNEL=$v timeout -k 10 400 python3 bench.py --config c5ggn --steps 2 --warmup 1 --no-cpu-baseline \
    > $O/c5ggn_v$v.json 2> $O/c5ggn_v$v.err || { echo "bench v$v failed"; tail -3 $O/c5ggn_v$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c5ggn_v$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('v$v', round(d['value'],4), r.get('kernel'), r.get('avg_ms'), d.get('parity_check',{}).get('pass'))"
done
