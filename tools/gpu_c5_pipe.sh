#!/bin/bash
# C5 pipelined LQN loop: parity tests, kernel-trace gap analysis, then same-box A/B against the
# HEAD build in _ab_old (and the cooperative direction + tail off).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/c5pipe
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sparse.py tests/test_gpu_default_path.py -m gpu -x -v --timeout 300 --timeout-method thread -k "lqn or c5 or sparse or LQN" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { # dir label env args
  (cd $1 && env $3 timeout -k 10 200 python3 bench.py --config c5 $4 --steps 50 --warmup 5 --no-cpu-baseline --no-check > /tmp/ab.log 2>&1) || exit 1
  tail -1 /tmp/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', round(d['value'],1), round(d['roofline']['avg_ms'],4))"
}
for rep in 1 2; do
  run _ab_old old-f64 "X=1" ""
  run . new-f64 "X=1" ""
  run . new-t1-f64 "SCS_BENCH_TIMING_EVERY=1" ""
  run _ab_old old-f32 "X=1" "--f32"
  run . new-f32 "X=1" "--f32"
done
bash tools/gpu_trace_c5.sh > $O/trace.log 2>&1 || { echo "trace failed"; tail -3 $O/trace.log; exit 1; }
head -16 gpurun_out/c5trace/gaps.txt
