#!/bin/bash
# chol probe + solver/sparse GPU tests + c2 and c5 bench lines
set -u
mkdir -p gpurun_out
timeout -k 10 120 ./build/probe_chol > gpurun_out/probe_chol.log 2>&1
rc=$?; echo "probe_chol rc=$rc"; cat gpurun_out/probe_chol.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -q -ra -k "cholesky or lu_fallback or sparse or synthetic" > gpurun_out/pytest_sc.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_sc.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for c in c2 c5; do
  timeout -k 10 600 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2> gpurun_out/bench_$c.err
  rc=$?; echo "bench $c rc=$rc"; tail -1 gpurun_out/bench_$c.log | cut -c1-1800; tail -3 gpurun_out/bench_$c.err
  [ $rc -eq 0 ] || exit $rc
done
