#!/bin/bash
# Cholesky: probe (OB / small-tile A/B), full GPU tests, C2 + C3 bench
set -u
mkdir -p gpurun_out
timeout -k 10 120 ./build/probe_chol_prof > gpurun_out/probe_chol_prof.log 2>&1; echo "prof rc=$?"; grep -E "phase|load" gpurun_out/probe_chol_prof.log
for cfg in "1 1024" "8 1024"; do
  set -- $cfg
  SCS_CHOL_OB=$1 SCS_GRAM_SMALL=$2 timeout -k 10 240 ./build/probe_chol > gpurun_out/probe_chol_ob$1_s$2.log 2>&1
  rc=$?; echo "probe_chol OB=$1 small=$2 rc=$rc"; grep -E "diag|factor|solve" gpurun_out/probe_chol_ob$1_s$2.log | sort -u
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_chol3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_chol3.log
[ $rc -eq 0 ] || exit $rc
summ() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get("roofline",{}); print(round(d["value"],4), "it/s", round(r.get("achieved",0),2), {k: round(v,2) for k,v in d["breakdown_ms_per_step"].items()})' $1; }
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/chol3_c2.log 2>&1; rc=$?; echo "c2 rc=$rc $(summ gpurun_out/chol3_c2.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > gpurun_out/chol3_c3.log 2>&1; rc=$?; echo "c3 rc=$rc $(summ gpurun_out/chol3_c3.log)"; [ $rc -eq 0 ] || exit $rc
