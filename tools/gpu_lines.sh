#!/bin/bash
# One bench line per configuration on the current build (default configuration, no env overrides):
# c2, c5 fp64 / fp32-stored / fp32 arithmetic, c5ggn, c4 at N = 2^19 with the cached Gram (c4 needs
# >= 4 GPUs at full size), c1; then the m = 8192 / 16384 factor kernel trace of the Cholesky probe.
#   usage: gpu_lines.sh [outdir]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/lines}; mkdir -p $O
line() { # label args...
  local l=$1; shift
  timeout -k 10 500 python3 bench.py "$@" > $O/$l.json 2> $O/$l.err || { echo "$l failed"; tail -3 $O/$l.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$l.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$l', round(d['value'],4), d['unit'], r.get('kernel'), r.get('bound'), round(r.get('frac',0),4), d.get('breakdown_ms_per_step'), (d.get('cpu_baseline') or {}).get('value'))"
}
line c2 --config c2 --steps 10 --warmup 2 && line c5 --config c5 && line c5_f32 --config c5 --f32 \
  && line c5_f32compute --config c5 --f32-compute && line c5ggn --config c5ggn --steps 2 --warmup 1 --no-cpu-baseline \
  && line c4half_cache --config c4 --N 524288 --gram-cache --steps 5 --warmup 1 --no-cpu-baseline \
  && line c1 --config c1 || exit 1
if [ -x ./tools/probes/bin/probe_chol_new ]; then
  T=$O/chol_trace; mkdir -p $T
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $T/rp -o run -- ./tools/probes/bin/probe_chol_new > $T/probe.log 2>&1 || { tail $T/probe.log; exit 1; }
  python3 tools/trace_chol_factor.py $T/rp/run_kernel_trace.csv > $T/trace_summary.txt && cat $T/trace_summary.txt
  rm -rf $T/rp
fi
