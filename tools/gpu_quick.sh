#!/bin/bash
# quick GPU loop: selected tests (-k expr in $1) + one bench config ($2)
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -ra -k "${1:-.}" > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_quick.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "${2:-}" ]; then
  timeout -k 10 900 python bench.py --config $2 --no-cpu-baseline > gpurun_out/bench_$2.log 2> gpurun_out/bench_$2.err
  rc=$?; echo "bench $2 rc=$rc"; tail -1 gpurun_out/bench_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('breakdown_ms_per_step'))"
fi
exit $rc
