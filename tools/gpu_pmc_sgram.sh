#!/bin/bash
# PMC passes (one counter group per run) over the C5-shaped ProxGGNSCORE step (bench.py --config c5ggn,
# one step) for the sparse Gram kernel; summarised by tools/pmc_summary_sgram.py.  Usage: gpu_pmc_sgram.sh [outdir]
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/pmc_sgram}; mkdir -p $O
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 400 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$name -o $name -- python3 bench.py --config c5ggn --steps 1 --warmup 0 --no-cpu-baseline > $O/$name.log 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run clk GRBM_GUI_ACTIVE SQ_BUSY_CYCLES
run fetch FETCH_SIZE
run write WRITE_SIZE
run tcc TCC_HIT_sum TCC_MISS_sum
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY
python3 tools/pmc_summary_sgram.py $O $O/summary.json
