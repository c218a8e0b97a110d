#!/bin/bash
# r06: the Cholesky chain's latency launches beside the bulk stream (m = 8192 probe factor): kernel traces and
# untraced factor times per arm (label=ENV ...), summarised by tools/trace_chain_wait.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${O:-gpurun_out/r06/chainwait}; mkdir -p $O
export PROBE_SIZES=${PROBE_SIZES:-8192}
for arm in "$@"; do
  label=${arm%%=*}; envs=${arm#*=}
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/$label -o run -- ./tools/probes/bin/probe_chol_new > $O/${label}_traced.log 2>&1 || { echo "$label traced failed"; tail -3 $O/${label}_traced.log; exit 1; }
  env $envs timeout -k 10 120 ./tools/probes/bin/probe_chol_new > $O/${label}_plain.log 2>&1 || { echo "$label failed"; exit 1; }
  echo "== $label ($envs): untraced $(grep factor $O/${label}_plain.log | tr '\n' ' ')"
  python3 tools/trace_chain_wait.py $O/$label/run_kernel_trace.csv || exit 1
done
