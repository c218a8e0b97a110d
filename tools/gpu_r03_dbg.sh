#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03dbg; mkdir -p $O
for i in 1 2; do timeout -k 10 300 python3 -u -m pytest -x -v --timeout 280 --timeout-method thread "tests/test_gpu_parity.py::test_step_grad_fx_keyword" "tests/test_gpu_shard.py" > $O/pytest$i.log 2>&1 || break; done
rc=$?; echo "pytest rc=$rc"; grep -E "^E .*(AssertionError|\(')" $O/pytest$i.log | head -5; tail -3 $O/pytest$i.log
