#!/bin/bash
# Launcher rehearsal on the one-GPU box, the driver's way (torch.distributed.run, 2 ranks) with the
# ranks sharing the GPU (--share-device --comm torch: gloo + the torch all-reduce callback), C3 shape
# at N = 2^17; then bench.py's own rank launcher (--gpus 2, no WORLD_SIZE).  Not a scaling number.
# Usage: gpu_r04_launcher.sh [outdir]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/launcher}; mkdir -p $O
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 2 --warmup 1 --config c3 --N 131072 --share-device --comm torch --no-cpu-baseline \
  > $O/torchrun_2.json 2> $O/torchrun_2.err || { tail -20 $O/torchrun_2.err; exit 1; }
tail -c 600 $O/torchrun_2.json; echo
timeout -k 10 400 python3 bench.py --gpus 2 --steps 2 --warmup 1 --config c3 --N 131072 --share-device --comm torch --no-cpu-baseline \
  > $O/self_2.json 2> $O/self_2.err || { tail -20 $O/self_2.err; exit 1; }
tail -c 600 $O/self_2.json; echo
