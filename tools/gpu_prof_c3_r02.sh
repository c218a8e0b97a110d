#!/bin/bash
# r02 C3 evidence: the default `python bench.py` line, then rocprofv3 kernel-trace stats and one PMC pass
# per counter group over the bench.  The profiled runs set SCS_CHOL_RESERVE_CUS=0: rocprofv3 segfaults at
# exit in a process that created a CU-masked stream (the factor's bulk stream at m <= 16384); the
# reserve touches only the solve's bulk stream, not the Gram these passes measure.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/prof_c3_r02
mkdir -p $O/stats $O/pmc
timeout -k 10 900 python3 bench.py > $O/bench_full.json 2> $O/bench_full.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -3 $O/bench_full.err; exit $rc; }
export SCS_CHOL_RESERVE_CUS=0
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/stats.log 2>&1
rc=$?; echo "rocprof stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 600 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/pmc/$name -o $name -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-check > $O/pmc/$name.log 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run clk GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES
run fetch FETCH_SIZE
run write WRITE_SIZE
run tcc TCC_HIT_sum TCC_MISS_sum
run sq SQ_INSTS_VALU_MFMA_F64 SQ_LDS_BANK_CONFLICT
python3 tools/pmc_summary.py $O/pmc $O/r02_gram_pmc.json --N 1048576 --m 16384 && cat $O/r02_gram_pmc.json
