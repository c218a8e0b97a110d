#!/bin/bash
# Segment records on 128-B lines (SCS_SPARSE_SEG_ALIGN, default) vs packed (0): the sparse GPU tests,
# then the C5-shaped sparse Gram time per launch (tools/sgram_diag.py, diag 0 is the production
# walk) in one process per setting, twice, and the c5ggn line.  Usage: gpu_r04_segalign.sh [outdir]
# (Run once with a build that had SCS_SPARSE_SEG_ALIGN -- records padded to 128-B lines; no gain,
# not kept: profiles/r04/segalign/.)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/segalign}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_sparse.py -x -v --timeout 300 --timeout-method thread > $O/pytest_sparse.log 2>&1 \
  || { tail -20 $O/pytest_sparse.log; exit 1; }
tail -2 $O/pytest_sparse.log
for r in 1 2; do
  for a in 0 1; do
    SCS_SPARSE_SEG_ALIGN=$a timeout -k 10 300 python3 -u tools/sgram_diag.py > $O/align${a}_r$r.log 2>&1 || { tail $O/align${a}_r$r.log; exit 1; }
    echo "== SCS_SPARSE_SEG_ALIGN=$a run $r"; grep "diag 0" $O/align${a}_r$r.log
  done
done
timeout -k 10 500 python3 bench.py --config c5ggn --steps 2 --warmup 1 --no-cpu-baseline > $O/c5ggn.json 2> $O/c5ggn.err || { tail -3 $O/c5ggn.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c5ggn.json').read().strip().splitlines()[-1]); print('c5ggn', round(d['value'],4), d.get('breakdown_ms_per_step'))"
