#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests -m gpu -q -ra > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for c in c1 c2 c3; do
  timeout -k 10 900 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2> gpurun_out/bench_$c.err
  rc=$?; echo "bench $c rc=$rc"; tail -1 gpurun_out/bench_$c.log | cut -c1-1500
  [ $rc -eq 0 ] || exit $rc
done
