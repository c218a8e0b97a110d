#!/bin/bash
# GPU suite (per-test timeout) + default bench line (C3, with CPU baseline)
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -ra --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_c3.log 2> gpurun_out/bench_c3.err
rc=$?; echo "bench rc=$rc"; tail -c 2500 gpurun_out/bench_c3.log; tail -3 gpurun_out/bench_c3.err
exit $rc
