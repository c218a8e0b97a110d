#!/bin/bash
# Gram kernel A/B: exactness checks (incl. bitwise pipe-vs-plain) + C3-size timing of the variants
set -u
mkdir -p gpurun_out
timeout -k 10 300 ./build/probe_gram > gpurun_out/probe_gram_small.log 2>&1
rc=$?; echo "probe small rc=$rc"; grep -E "CHECK|GRAM" gpurun_out/probe_gram_small.log
[ $rc -eq 0 ] || exit $rc
GRAM_EXPERIMENTS=1 timeout -k 10 400 ./build/probe_gram 1048576 16384 1 > gpurun_out/probe_gram_c3.log 2>&1
rc=$?; echo "probe c3 rc=$rc"; cat gpurun_out/probe_gram_c3.log
exit $rc
