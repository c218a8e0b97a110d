#!/bin/bash
# bench lines for every single-GPU config (no CPU baselines)
set -u
mkdir -p gpurun_out
for c in c1 c3 c2 c5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/benchall_$c.log 2> gpurun_out/benchall_$c.err
  rc=$?; echo "$c rc=$rc"; tail -1 gpurun_out/benchall_$c.log | cut -c1-400; [ $rc -eq 0 ] || { tail -5 gpurun_out/benchall_$c.err; exit $rc; }
done
