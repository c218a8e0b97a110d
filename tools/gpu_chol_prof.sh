#!/bin/bash
# diagonal-kernel phase profile (probe_chol_prof) and factor timings, both diagonal schedules
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/cholprof
mkdir -p $O
for d in 0 1; do
  SCS_CHOL_DIAG=$d timeout -k 10 120 ./tools/probes/bin/probe_chol_prof > $O/prof_d$d.log 2>&1 || { echo "prof failed"; tail $O/prof_d$d.log; exit 1; }
  echo "== diag=$d"; cat $O/prof_d$d.log
done
