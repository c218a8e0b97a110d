#!/bin/bash
# rocprofv3 kernel stats of probe_chol at OB=1 and OB=8
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for ob in 1 8; do
  SCS_CHOL_OB=$ob timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_chol_ob$ob -o run -- ./build/probe_chol > gpurun_out/prof_chol_ob$ob.log 2>&1
  rc=$?; echo "OB=$ob rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/prof_chol_ob$ob -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -12
done
