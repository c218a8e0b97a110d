#!/bin/bash
# Parameterised A/B runner (replaces round 4's one-off tools/gpu_r04_*.sh; the git history keeps them).
# Runs one command under several environment settings, the settings interleaved over R rounds (box
# drift lands on every arm alike), each run under its own time limit; greps one result line per run.
#
#   tools/gpu_ab.sh OUTDIR ROUNDS 'COMMAND' 'GREP' LABEL='ENV=V ENV2=W' LABEL2='...' ...
#
# e.g. the factor probe at two outer-block sizes:
#   tools/gpu_ab.sh gpurun_out/r05/ob 2 './tools/probes/bin/probe_chol_new' 'factor' ob4='SCS_CHOL_OB=4' ob8='SCS_CHOL_OB=8'
# or two bench lines:
#   tools/gpu_ab.sh gpurun_out/r05/c2 2 'python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --no-check' \
#       '"value"' base='' nosplit='SCS_CHOL_C12_SPLIT=0'
# A failing run ends the script (no retries); per-run logs are OUTDIR/<label>_r<round>.log.
set -o pipefail
O=$1; R=$2; CMD=$3; PAT=$4; shift 4
[ -n "$O" ] && [ -n "$R" ] && [ -n "$CMD" ] && [ $# -ge 1 ] || { echo "usage: $0 OUTDIR ROUNDS CMD GREP LABEL=ENV..." >&2; exit 2; }
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p "$O"
TL=${AB_TIMEOUT:-300}
for r in $(seq 1 "$R"); do
  for arm in "$@"; do
    label=${arm%%=*}; envs=${arm#*=}
    log="$O/${label}_r$r.log"
    env $envs timeout -k 10 "$TL" bash -c "$CMD" > "$log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$label r$r: rc=$rc"; tail -5 "$log"; exit $rc; fi
    echo "$label r$r: $(grep -- "$PAT" "$log" | tail -1 | cut -c1-400)"
  done
done
