#!/bin/bash
# r02 C5 evidence: fp64 / fp32 bench lines under rocprofv3 --kernel-trace --stats (SpMV avg from rocprof
# vs the bench's sampled hipEvents)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/prof_c5
mkdir -p $O
for arm in f64 f32; do
  a=""; [ $arm = f32 ] && a="--f32"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/rp_$arm -o run --output-format csv -- python3 bench.py --config c5 $a > $O/bench_$arm.log 2>&1 || { echo "rocprof $arm failed"; tail -3 $O/bench_$arm.log; exit 1; }
  grep '^{' $O/bench_$arm.log | tail -1 > $O/bench_$arm.json
  python3 -c "import json; d=json.loads(open('$O/bench_$arm.json').read()); r=d['roofline']; print('$arm', round(d['value'],1), round(r['avg_ms'],4), round(r['frac'],3), (d.get('cpu_baseline') or {}).get('value'))"
  f=$(find $O/rp_$arm -name '*kernel_stats.csv' | head -1)
  grep -i spmv "$f" | cut -d, -f1-4
done
