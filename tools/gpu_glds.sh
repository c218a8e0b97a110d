#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "gram or synthetic or shard or group" > gpurun_out/pytest_glds.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_glds.log
[ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  SCS_GRAM_GLDS=$v timeout -k 10 600 python bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_c3_glds$v.log 2> gpurun_out/bench_c3_glds$v.err
  rc=$?; echo "c3 glds=$v rc=$rc $(tail -1 gpurun_out/bench_c3_glds$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"],4), round(r["achieved"],2), d["breakdown_ms_per_step"])')"
  [ $rc -eq 0 ] || exit $rc
done
