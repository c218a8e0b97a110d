#!/bin/bash
# Interleaved-schedule Gram kernel: bitwise vs the register-staged kernel + timing
set -u
mkdir -p gpurun_out
for sz in "48 256 1" "1040 384 1" "4096 1024 1"; do
  GRAM_SIA=1 timeout -k 10 60 ./build/probe_gram $sz > gpurun_out/sia_small.log 2>&1 || { echo "small $sz failed rc=$?"; cat gpurun_out/sia_small.log; exit 1; }
  grep -E "CHECK sia|SIA" gpurun_out/sia_small.log
done
GRAM_SIA=1 timeout -k 10 200 ./build/probe_gram 262144 16384 2 > gpurun_out/sia_big.log 2>&1
rc=$?; grep -E "CHECK sia|SIA|GRAM" gpurun_out/sia_big.log; exit $rc
