#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 120 ./build/probe_chol_prof > gpurun_out/probe_chol_prof.log 2>&1
rc=$?; echo "probe_chol_prof rc=$rc"; cat gpurun_out/probe_chol_prof.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "cholesky or lu_fallback or synthetic or reference or group" > gpurun_out/pytest_chol.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_chol.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config c2 --no-cpu-baseline > gpurun_out/bench_c2.log 2> gpurun_out/bench_c2.err
rc=$?; echo "bench c2 rc=$rc"; tail -1 gpurun_out/bench_c2.log | cut -c1-300; tail -1 gpurun_out/bench_c2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["breakdown_ms_per_step"])'
