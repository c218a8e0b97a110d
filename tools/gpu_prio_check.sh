set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06/prio_c2
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "cholesky or chol or default_path or solve or lookahead or superblock" > gpurun_out/r06/prio_c2/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r06/prio_c2/pytest.log; [ $rc -eq 0 ] || exit $rc
AB_TIMEOUT=300 bash tools/gpu_ab.sh gpurun_out/r06/prio_c2 2 'python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --no-check' '"value"' prio="" base="SCS_CHOL_PRIO=0" > gpurun_out/r06/prio_c2/ab.txt 2>&1; rc=$?
for f in gpurun_out/r06/prio_c2/*_r*.log; do tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value'],3), {k: round(v,2) for k,v in d['breakdown_ms_per_step'].items()})"; done
exit $rc
