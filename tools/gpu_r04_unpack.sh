#!/bin/bash
# The exchange path's pack / unpack as LDS-tiled transposes: the exchange tests (forced exchange
# bit-identical, shards, multi-device groups, sparse) and the C3 per-rank shape with and without the
# exchange path, twice.  Usage: gpu_r04_unpack.sh [outdir]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/unpack}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_comm.py tests/test_gpu_shard.py tests/test_gpu_multi.py tests/test_gpu_sparse.py \
  -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for f in "" "--force-comm"; do
    timeout -k 10 300 python3 bench.py --config c3 --N 131072 --steps 3 --warmup 1 --no-cpu-baseline --no-check $f > $O/run.json 2> $O/run.err || { tail -3 $O/run.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/run.json').read().strip().splitlines()[-1]); print('force=$f', d['breakdown_ms_per_step'], round(d['ms_per_step'], 2))"
  done
done
