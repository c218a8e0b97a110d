#!/bin/bash
# bench lines (with CPU baselines) for every single-GPU config; C4 at half size (N = 2^19) in
# both modes -- the full C4 needs >= 4 GPUs
set -u
mkdir -p gpurun_out
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/benchall_$tag.log 2> gpurun_out/benchall_$tag.err
  local rc=$?; echo "$tag rc=$rc"; tail -1 gpurun_out/benchall_$tag.log | cut -c1-300
  [ $rc -eq 0 ] || { tail -5 gpurun_out/benchall_$tag.err; exit $rc; }
}
run c1 --config c1
run c2 --config c2
run c5 --config c5
run c5f32 --config c5 --f32
run c4half --config c4 --N 524288 --steps 3 --warmup 1
run c4half_cache --config c4 --N 524288 --steps 5 --warmup 1 --gram-cache
