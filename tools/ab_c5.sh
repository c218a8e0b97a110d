set -o pipefail
mkdir -p gpurun_out
run() { # dir label args
  (cd $1 && timeout -k 10 200 python3 bench.py --config c5 $3 --steps 30 --warmup 3 --no-cpu-baseline --no-check > /tmp/ab.log 2>&1) || exit 1
  tail -1 /tmp/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', round(d['value'],1), round(d['roofline']['avg_ms'],4))"
}
for rep in 1 2; do
  run _ab_old old-f64 ""
  run . new-f64 ""
  run _ab_old old-f32 "--f32"
  run . new-f32 "--f32"
done
