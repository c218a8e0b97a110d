#!/bin/bash
# two-operand Gram launches (strip solves, LU TRSM / updates) on the interleaved kernel: tests, then
# C4-half cached solve, C2, and the LU timing tool with SCS_GRAM_GEN2=0 / default
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/gen2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lu.py tests/test_gpu_default_path.py -m gpu -x -v --timeout 300 --timeout-method thread -k "cholesky or blocked or indefinite or lu or LU or c4 or sample" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for g in 0 1; do
  SCS_GRAM_GEN2=$g timeout -k 10 300 python3 bench.py --config c4 --N 524288 --gram-cache --steps 2 --warmup 1 --no-cpu-baseline --no-check > $O/c4_g$g.json 2> $O/c4_g$g.err || { echo "bench failed"; tail -3 $O/c4_g$g.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_g$g.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c4 gen2=$g', round(d['value'],4), round(r['avg_ms'],2), round(r['frac'],3))"
  SCS_GRAM_GEN2=$g timeout -k 10 300 python3 bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-check > $O/c2_g$g.json 2> $O/c2_g$g.err || { echo "bench failed"; tail -3 $O/c2_g$g.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c2_g$g.json').read().strip().splitlines()[-1]); print('c2 gen2=$g', round(d['value'],4), d['breakdown_ms_per_step'])"
  SCS_GRAM_GEN2=$g timeout -k 10 300 python3 tools/lu_time.py > $O/lu_g$g.txt 2>&1 || { echo "lu_time failed"; tail -3 $O/lu_g$g.txt; exit 1; }
  echo "lu gen2=$g"; tail -3 $O/lu_g$g.txt
done
