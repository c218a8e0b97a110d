#!/bin/bash
# r03 C3 evidence on the DEFAULT configuration (no env overrides): the default `python bench.py` line,
# rocprofv3 kernel-trace stats of a 2-step run, one PMC pass per counter group over a 1-step run
# (summarised by tools/pmc_summary.py into r03_gram_pmc.json), then the default line again with that
# PMC record in place (roofline.traffic).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03c3
mkdir -p $O/pmc
timeout -k 10 900 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -3 $O/bench_default.err; exit $rc; }
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/stats.log 2>&1
rc=$?; echo "rocprof stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/rocpd_stats.py $O/stats/run_results.db --csv $O/c3_kernel_stats.csv > /dev/null || exit 1
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
python3 tools/pmc_summary.py $O/pmc $O/r03_gram_pmc.json --N 1048576 --m 16384 && cat $O/r03_gram_pmc.json || exit 1
cp $O/r03_gram_pmc.json profiles/r03_gram_pmc.json
timeout -k 10 900 python3 bench.py > $O/bench_default_traffic.json 2> $O/bench_default_traffic.err
rc=$?; echo "bench (traffic) rc=$rc"; tail -c 600 $O/bench_default_traffic.json
