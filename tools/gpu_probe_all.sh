#!/bin/bash
# probes (gram square vs tall, chol) then the solver/sparse/synthetic GPU tests and c2/c3/c5 bench lines
set -u
mkdir -p gpurun_out
timeout -k 10 300 ./build/probe_gram > gpurun_out/probe_gram.log 2>&1
rc=$?; echo "probe_gram rc=$rc"; cat gpurun_out/probe_gram.log
[ $rc -eq 0 ] || exit $rc
GRAM_EXPERIMENTS=1 timeout -k 10 300 ./build/probe_gram 1048576 16384 2 > gpurun_out/probe_gram_c3.log 2>&1
rc=$?; echo "probe_gram c3 rc=$rc"; cat gpurun_out/probe_gram_c3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./build/probe_chol > gpurun_out/probe_chol.log 2>&1
rc=$?; echo "probe_chol rc=$rc"; cat gpurun_out/probe_chol.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -q -ra -k "cholesky or lu_fallback or sparse or synthetic or gram or shard or two_loop" > gpurun_out/pytest_sc.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_sc.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for c in c2 c5 c3; do
  timeout -k 10 600 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2> gpurun_out/bench_$c.err
  rc=$?; echo "bench $c rc=$rc"; tail -1 gpurun_out/bench_$c.log | cut -c1-1800; tail -3 gpurun_out/bench_$c.err
  [ $rc -eq 0 ] || exit $rc
done
