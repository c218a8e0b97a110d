#!/bin/bash
# r04 batch 3: the group abort-path test, a host-exchange group rehearsal line (4 sub-contexts on one GPU,
# C3 shape at N = 2^17), the C5-shaped GGN line on the default sparse Gram (variant 8) and its PMC passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/batch3}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_multi.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider -k "fault or host_exchange" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --single-process --gpus 4 --device-exchange host --N 131072 --steps 3 --warmup 1 \
  --no-cpu-baseline > $O/bench_c3_group4_host.json 2> $O/bench_c3_group4_host.err || { tail -5 $O/bench_c3_group4_host.err; exit 1; }
tail -c 900 $O/bench_c3_group4_host.json; echo
timeout -k 10 400 python3 bench.py --config c5ggn --steps 2 --warmup 1 --no-cpu-baseline > $O/c5ggn.json 2> $O/c5ggn.err \
  || { tail -3 $O/c5ggn.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c5ggn.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c5ggn', round(d['value'],4), r.get('kernel'), r.get('avg_ms'), r.get('frac'), d.get('breakdown_ms_per_step'))"
bash tools/gpu_pmc_sgram.sh $O/pmc_sgram
