#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests -m gpu -q -ra > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
GRAM_EXPERIMENTS=1 timeout -k 10 400 ./build/probe_gram 1048576 16384 1 > gpurun_out/gram_exp3.log 2>&1
rc=$?; echo "probe rc=$rc"; cat gpurun_out/gram_exp3.log
exit $rc
