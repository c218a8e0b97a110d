#!/bin/bash
# Sparse Gram flat-issue kernel (variant 6) vs r03's variant 5 (tests + C5-shaped GGN bench), then the
# m = 8192 / 16384 factor kernel trace (C12 split) kept as CSV for tools/trace_chol_factor.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/sg}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_sparse.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "gram" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 5 6; do
  SCS_SPARSE_GRAM_KERNEL=$v timeout -k 10 400 python3 bench.py --config c5ggn --steps 2 --warmup 1 --no-cpu-baseline \
    > $O/c5ggn_v$v.json 2> $O/c5ggn_v$v.err || { echo "bench v$v failed"; tail -3 $O/c5ggn_v$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c5ggn_v$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('v$v', round(d['value'],4), r.get('kernel'), r.get('avg_ms'), r.get('frac'), d.get('breakdown_ms_per_step'), d.get('parity_check',{}).get('pass'))"
done
T=$O/chol_trace; mkdir -p $T
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $T/rp -o run -- ./tools/probes/bin/probe_chol_c12 > $T/probe.log 2>&1 || { tail $T/probe.log; exit 1; }
python3 tools/trace_chol_factor.py $T/rp/run_kernel_trace.csv > $T/trace_summary.txt && cat $T/trace_summary.txt
