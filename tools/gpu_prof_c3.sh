#!/bin/bash
# C3 bench line (with cpu_baseline) + rocprofv3 kernel-trace stats + PMC passes on the bench itself
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_c3 gpurun_out/pmc_c3
timeout -k 10 900 python bench.py > gpurun_out/bench_full.log 2> gpurun_out/bench_full.err
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_full.log | cut -c1-600
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1
rc=$?; echo "rocprof stats rc=$rc"; tail -1 gpurun_out/prof_c3.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 600 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc_c3/$name -o $name -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_c3/$name.log 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run clk GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES
run fetch FETCH_SIZE
run write WRITE_SIZE
run tcc TCC_HIT_sum TCC_MISS_sum
run sq SQ_INSTS_VALU_MFMA_F64 SQ_LDS_BANK_CONFLICT
find gpurun_out/prof_c3 gpurun_out/pmc_c3 -name "*.csv" | head -20
