#!/bin/bash
# Gram pipe in the library: gram/parity tests, C3 bench, C2 bench square vs tall(pipe)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gram or synthetic or ggn or nscore" > gpurun_out/pytest_ab2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab2.log
[ $rc -eq 0 ] || exit $rc
summ() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get("roofline",{}); print(round(d["value"],4), "it/s", round(r.get("achieved",0),2), {k: round(v,2) for k,v in d["breakdown_ms_per_step"].items()})' $1; }
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > gpurun_out/ab2_c3.log 2>&1; rc=$?; echo "c3 rc=$rc $(summ gpurun_out/ab2_c3.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/ab2_c2.log 2>&1; rc=$?; echo "c2 rc=$rc $(summ gpurun_out/ab2_c2.log)"; [ $rc -eq 0 ] || exit $rc
SCS_GRAM_TALL=1 timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/ab2_c2t.log 2>&1; rc=$?; echo "c2 tall rc=$rc $(summ gpurun_out/ab2_c2t.log)"; [ $rc -eq 0 ] || exit $rc
