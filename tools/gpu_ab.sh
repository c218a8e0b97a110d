#!/bin/bash
# GPU tests (broad subset) + bench A/B of env toggles
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -ra > gpurun_out/pytest_all.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_all.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run() {  # name env... -- args
  local name=$1; shift
  env "$@" timeout -k 10 600 python bench.py --no-cpu-baseline $BARGS > gpurun_out/ab_$name.log 2> gpurun_out/ab_$name.err
  local rc=$?
  echo "$name rc=$rc $(tail -1 gpurun_out/ab_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d.get("roofline",{}); print(round(d["value"],4), "it/s", round(d["ms_per_step"],2), "ms", r.get("kernel"), round(r.get("achieved",0),2), r.get("unit"), {k: round(v,2) for k,v in d["breakdown_ms_per_step"].items()})' 2>&1)"
  return $rc
}
BARGS="--config c5" run c5 X=1 || exit 1
BARGS="--config c2" run c2_sched X=1 || exit 1
BARGS="--config c2" run c2_nosched SCS_GRAM_SCHED=0 || exit 1
BARGS="--config c2" run c2_square SCS_GRAM_TALL=0 || exit 1
BARGS="--config c3" run c3_sched X=1 || exit 1
BARGS="--config c3" run c3_square SCS_GRAM_TALL=0 || exit 1
