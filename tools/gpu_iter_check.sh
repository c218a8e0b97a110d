#!/bin/bash
# GPU tests + C5 bench + C5 kernel trace (host gaps per step)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/iter
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/iter/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/iter/pytest.log; exit 1; }
tail -1 gpurun_out/iter/pytest.log
for f in "" "--f32"; do
timeout -k 10 300 python3 bench.py --config c5 $f --no-cpu-baseline > gpurun_out/iter/c5$f.json 2> gpurun_out/iter/c5$f.err || { tail gpurun_out/iter/c5$f.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/iter/c5$f.json').read().strip().splitlines()[-1]); print('c5 $f', d['value'], d['breakdown_ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/iter/rp -o run -- python3 bench.py --config c5 --no-cpu-baseline > gpurun_out/iter/rp.log 2>&1 || { tail gpurun_out/iter/rp.log; exit 1; }
echo done
