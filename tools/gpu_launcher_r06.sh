#!/bin/bash
# r06 launcher rehearsal on the one-GPU box, the driver's way (torch.distributed.run) with 4 and 8 ranks sharing
# the GPU (--share-device --comm torch: gloo + the torch all-reduce callback), C3 shape at N = 2^17 in total.
# Not a scaling number: it exercises the rank plumbing, the row split, the exchange and verify_ranks at world 4 / 8.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r06/launcher}; mkdir -p $O
for n in 4 8; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2953$n \
    bench.py --gpus $n --steps 2 --warmup 1 --config c3 --N 131072 --share-device --comm torch --no-cpu-baseline \
    > $O/torchrun_$n.json 2> $O/torchrun_$n.err || { tail -20 $O/torchrun_$n.err; exit 1; }
  tail -1 $O/torchrun_$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['n_gpus'], d['value'], d.get('ranks_consistent'), d.get('parity_check', {}).get('pass'), [ (r['rank'], r['rows']) for r in d.get('ranks', [])])"
done
