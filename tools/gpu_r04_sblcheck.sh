#!/bin/bash
# After the super-block bulk order became the default: the Cholesky GPU tests, the C5-shaped GGN
# line (m = 65536 factor), the C4-half cached-Gram line (m = 32768) and the bulk-launch efficiency
# trace at m = 65536.  Usage: gpu_r04_sblcheck.sh [outdir]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/sblcheck}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "cholesky" > $O/pytest_chol.log 2>&1 \
  || { tail -20 $O/pytest_chol.log; exit 1; }
tail -3 $O/pytest_chol.log
line() { # label args...
  local l=$1; shift
  timeout -k 10 500 python3 bench.py "$@" > $O/$l.json 2> $O/$l.err || { echo "$l failed"; tail -3 $O/$l.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$l.json').read().strip().splitlines()[-1]); print('$l', round(d['value'],4), d['unit'], d.get('breakdown_ms_per_step'))"
}
line c5ggn --config c5ggn --steps 2 --warmup 1 --no-cpu-baseline && line c4half_cache --config c4 --N 524288 --gram-cache --steps 5 --warmup 1 --no-cpu-baseline || exit 1
PROBE_SIZES=65536 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o run -- ./tools/probes/bin/probe_chol_sz > $O/probe.log 2>&1 || { tail $O/probe.log; exit 1; }
python3 tools/trace_bulk_eff.py $O/rp/run_kernel_trace.csv 65536 > $O/bulk_eff_m65536.txt && cat $O/bulk_eff_m65536.txt
rm -rf $O/rp
