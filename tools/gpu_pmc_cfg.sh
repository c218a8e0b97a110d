#!/bin/bash
# PMC passes (one counter group per run) of the Gram kernel over `bench.py $@ --steps 1 --warmup 0`
# into gpurun_out/pmc_cfg/<group>/ (summarise with tools/pmc_summary.py)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc_cfg
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc_cfg/$name -o $name -- python3 bench.py $ARGS --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_cfg/$name.log 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
ARGS="$*"
run clk GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES
run fetch FETCH_SIZE
run write WRITE_SIZE
run tcc TCC_HIT_sum TCC_MISS_sum
run sq SQ_INSTS_VALU_MFMA_F64 SQ_LDS_BANK_CONFLICT
