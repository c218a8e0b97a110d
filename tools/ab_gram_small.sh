#!/bin/bash
# SCS_GRAM_SMALL = 64 (old default) vs 128 on the other users of the latency kernel: the m = 32768 cached-Gram
# solve (C4 at N = 2^19), the LU (n = 8192) and the reference-mode QR (n = 8192), alternated on one box
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/gsmall; mkdir -p $O
for v in 64 128; do
  SCS_GRAM_SMALL=$v timeout -k 10 400 python3 bench.py --config c4 --N 524288 --gram-cache --steps 4 --warmup 1 --no-cpu-baseline --no-check > $O/c4_$v.json 2> $O/c4_$v.err || { tail -3 $O/c4_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_$v.json').read().strip().splitlines()[-1]); print('c4half cache small $v', round(d['value'],4), round(d['breakdown_ms_per_step']['solve'],2))"
  SCS_GRAM_SMALL=$v timeout -k 10 300 python3 tools/lu_time.py 8192 > $O/lu_$v.log 2>&1 || { tail -3 $O/lu_$v.log; exit 1; }
  echo "lu small $v: $(tail -1 $O/lu_$v.log | cut -c1-160)"
  SCS_GRAM_SMALL=$v timeout -k 10 300 python3 tools/qr_time.py 8192 > $O/qr_$v.log 2>&1 || { tail -3 $O/qr_$v.log; exit 1; }
  echo "qr small $v: $(tail -2 $O/qr_$v.log | tr '\n' ' ' | cut -c1-200)"
done
