#!/bin/bash
# full GPU suite + c2/c3/c5 bench lines (no CPU baseline)
set -u
mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests -m gpu -q -ra > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for c in c3 c2 c5; do
  timeout -k 10 600 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2> gpurun_out/bench_$c.err
  rc=$?; echo "bench $c rc=$rc $(tail -1 gpurun_out/bench_$c.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d.get("roofline",{}); print(round(d["value"],4), "it/s", r.get("kernel"), round(r.get("achieved",0),2), r.get("unit"), {k: round(v,2) for k,v in d["breakdown_ms_per_step"].items()}, "hbm_stream", round(d.get("hbm_gbs_streaming",0)))' 2>&1)"
  [ $rc -eq 0 ] || exit $rc
done
