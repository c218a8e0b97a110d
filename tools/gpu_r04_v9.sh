#!/bin/bash
# Variant 9 of the sparse Gram (two rows per load instruction): the sparse GPU tests (bitwise vs
# variant 8 and the others), the timing builds + both variants at the C5 shape (tools/sgram_diag.py),
# and the c5ggn line under each.  Usage: gpu_r04_v9.sh [outdir]
# (Run twice with builds that had a variant 9, sparse_gram_seg2_kernel -- three half-wave atomics per
# row pair, then v_permlane32_swap -- both bitwise equal to variant 8 and slower (646 / 570 vs 539 ms),
# dropped: profiles/r04/v9/, v9b/.)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/v9}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_sparse.py -x -v --timeout 300 --timeout-method thread > $O/pytest_sparse.log 2>&1 \
  || { tail -20 $O/pytest_sparse.log; exit 1; }
tail -2 $O/pytest_sparse.log
timeout -k 10 400 python3 -u tools/sgram_diag.py > $O/diag.log 2>&1 || { tail $O/diag.log; exit 1; }
cat $O/diag.log
for v in 8 9; do
  SCS_SPARSE_GRAM_KERNEL=$v timeout -k 10 500 python3 bench.py --config c5ggn --steps 2 --warmup 1 --no-cpu-baseline > $O/c5ggn_v$v.json 2> $O/c5ggn_v$v.err || { tail -3 $O/c5ggn_v$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c5ggn_v$v.json').read().strip().splitlines()[-1]); print('c5ggn v$v', round(d['value'],4), d.get('breakdown_ms_per_step'), (d.get('roofline') or {}).get('kernel'))"
done
