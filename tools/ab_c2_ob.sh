#!/bin/bash
# C2 bench lines with the default outer block (4 at m = 8192) against SCS_CHOL_OB=8, alternated on one box,
# then the factor tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/c2ob; mkdir -p $O
run() { # label env
  env $2 timeout -k 10 300 python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --no-check > $O/$1.json 2> $O/$1.err || { tail -3 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', round(d['value'],3), {k: round(v,2) for k,v in d['breakdown_ms_per_step'].items()})"
}
for rep in 1 2; do run ob4_$rep SCS_CHOL_OBX=0; run ob8_$rep SCS_CHOL_OB=8; done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "cholesky or chol or default_path or solve or qr or lu" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest.log; exit $rc
