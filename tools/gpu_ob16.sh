#!/bin/bash
# 16-block outer steps at m = 32768: Cholesky tests, then the C4-half cached-Gram solve (OB 8 vs default)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/ob16
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_default_path.py -m gpu -x -v --timeout 300 --timeout-method thread -k "cholesky or blocked or c4 or C4" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for ob in 8 16; do
  SCS_CHOL_OB=$ob timeout -k 10 300 python3 bench.py --config c4 --N 524288 --gram-cache --steps 2 --warmup 1 --no-cpu-baseline --no-check > $O/c4_ob$ob.json 2> $O/c4_ob$ob.err || { echo "bench failed"; tail -3 $O/c4_ob$ob.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_ob$ob.json').read().strip().splitlines()[-1]); r=d['roofline']; print('ob=$ob', round(d['value'],4), round(r['avg_ms'],2), round(r['frac'],3))"
done
