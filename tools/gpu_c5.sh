#!/bin/bash
# C5: sparse tests + bench (fp64, fp32 values)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sparse or lqn or c5" > gpurun_out/pytest_c5.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_c5.log
[ $rc -eq 0 ] || exit $rc
summ() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get("roofline",{}); print(round(d["value"],2), "it/s", round(r.get("achieved",0),1), r.get("unit"), round(r.get("avg_ms",0),3), "ms", {k: round(v,3) for k,v in d["breakdown_ms_per_step"].items()})' $1; }
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/c5.log 2>&1; rc=$?; echo "c5 rc=$rc $(summ gpurun_out/c5.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c5 --f32 --no-cpu-baseline > gpurun_out/c5f.log 2>&1; rc=$?; echo "c5 f32 rc=$rc $(summ gpurun_out/c5f.log)"; [ $rc -eq 0 ] || exit $rc
