#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 120 ./build/probe_chol_prof > gpurun_out/probe_chol_prof.log 2>&1
rc=$?; echo "probe_chol_prof rc=$rc"; cat gpurun_out/probe_chol_prof.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests/test_gpu_sparse.py -q -x > gpurun_out/pytest_sparse.log 2>&1
rc=$?; echo "pytest sparse rc=$rc"; tail -2 gpurun_out/pytest_sparse.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config c5 > gpurun_out/bench_c5.log 2> gpurun_out/bench_c5.err
rc=$?; echo "bench c5 rc=$rc"; tail -1 gpurun_out/bench_c5.log | cut -c1-2500
timeout -k 10 600 python bench.py --config c5 --f32 --no-cpu-baseline > gpurun_out/bench_c5f32.log 2> gpurun_out/bench_c5f32.err
rc=$?; echo "bench c5 f32 rc=$rc"; tail -1 gpurun_out/bench_c5f32.log | cut -c1-1500
