#!/bin/bash
# PMC passes (one counter group per run) over the C2 bench for its Gram kernel -> tools/pmc_summary.py
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc_c2
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc_c2/$name -o $name -- python3 bench.py --config c2 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_c2/$name.log 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run clk GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES
run fetch FETCH_SIZE
run write WRITE_SIZE
run tcc TCC_HIT_sum TCC_MISS_sum
run sq SQ_INSTS_VALU_MFMA_F64 SQ_LDS_BANK_CONFLICT
python3 tools/pmc_summary.py gpurun_out/pmc_c2 gpurun_out/pmc_c2/r01_gram_pmc_c2.json --N 100000 --m 8192 && cat gpurun_out/pmc_c2/r01_gram_pmc_c2.json
