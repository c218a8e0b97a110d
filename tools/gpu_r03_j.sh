#!/bin/bash
# r03: the latency-overlapped sparse Gram -- tests (bit identity with the previous kernel), then the
# C5-shaped ProxGGNSCORE step with each kernel, then rocprofv3 kernel stats of the default.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03j; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_sparse.py::test_sparse_gram_priced_by_nnz" \
  > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest.log | tail -2; [ $rc -eq 0 ] || exit $rc
b() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --config c5ggn --steps 2 --warmup 1 --no-cpu-baseline > $O/$n.log 2>&1 \
    || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['value'],4), d['breakdown_ms_per_step'], d['roofline']['kernel'])"
}
b pipe
b r64 SCS_SPARSE_GRAM_KERNEL=3
b bmaj32 SCS_SPARSE_GRAM_KERNEL=4
b bmaj64 SCS_SPARSE_GRAM_KERNEL=5
b v1 SCS_SPARSE_GRAM_KERNEL=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/rp -o run -- python3 bench.py --config c5ggn --steps 1 --warmup 0 \
  --no-cpu-baseline --no-check > $O/rp.log 2>&1; echo "rocprof rc=$?"
python3 tools/rocpd_stats.py $O/rp/run_results.db --csv $O/c5ggn_stats.csv > /dev/null && head -4 $O/c5ggn_stats.csv | cut -c1-60,150-
