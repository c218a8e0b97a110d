#!/bin/bash
# GPU validation run (used with gpurun): parity tests, smoke, a short bench.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -ra > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --N 131072 --m 4096 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_small.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench_small.log
exit $rc
