#!/bin/bash
# r03: the sparse Gram default (64 rows per batch, b-major items) -- sparse GPU tests, the c5ggn line,
# and its rocprofv3 kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sparse.py \
  > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --config c5ggn --steps 3 --warmup 1 > $O/c5ggn.log 2>&1 || { echo bench failed; tail -5 $O/c5ggn.log; exit 1; }
grep '^{' $O/c5ggn.log | tail -1 > $O/c5ggn.json
python3 -c "import json; d=json.load(open('$O/c5ggn.json')); print(round(d['value'],4), d['breakdown_ms_per_step'], d['roofline']['kernel'], d.get('cpu_baseline'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/rp -o run -- python3 bench.py --config c5ggn --steps 1 --warmup 0 \
  --no-cpu-baseline --no-check > $O/rp.log 2>&1; echo "rocprof rc=$?"
python3 tools/rocpd_stats.py $O/rp/run_results.db --csv $O/c5ggn_stats.csv > /dev/null && head -4 $O/c5ggn_stats.csv | cut -c1-70,150-
