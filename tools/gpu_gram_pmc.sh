#!/bin/bash
# Headline-Gram evidence on the DEFAULT configuration (no env overrides): rocprofv3 kernel-trace stats
# of a 2-step C3 run, then one PMC pass per counter group over a 1-step run (summarised by
# tools/pmc_summary.py into profiles/<tag>_gram_pmc.json, which bench.py reads for roofline.traffic
# when the record's kernel name equals the kernel the run launched).
#   usage: tools/gpu_gram_pmc.sh <tag>        e.g. r05
set -u
TAG=${1:?tag}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG}_gram
mkdir -p $O/pmc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/stats.log 2>&1
rc=$?; echo "rocprof stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/rocpd_stats.py $O/stats/run_results.db --csv $O/c3_kernel_stats.csv > /dev/null || exit 1
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/pmc/$name -o $name -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-check > $O/pmc/$name.log 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run clk GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES
run fetch FETCH_SIZE
run write WRITE_SIZE
run tcc TCC_HIT_sum TCC_MISS_sum
run sq SQ_INSTS_VALU_MFMA_F64 SQ_LDS_BANK_CONFLICT
python3 tools/pmc_summary.py $O/pmc $O/${TAG}_gram_pmc.json --N 1048576 --m 16384 > /dev/null || exit 1
echo done
