cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/c3_end; mkdir -p $O
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/stats.log 2>&1
rc=$?; echo "rocprof stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/rocpd_stats.py $O/stats/run_results.db --csv $O/c3_kernel_stats.csv > /dev/null || exit 1
grep '"metric"' $O/stats.log | tail -1 > $O/bench_c3_under_rocprof.json
head -8 $O/c3_kernel_stats.csv | cut -c1-160
python3 -c "import json; d=json.load(open('$O/bench_c3_under_rocprof.json')); print('bench hipEvent Gram avg ms', d['roofline']['avg_ms'], 'value', d['value'])"
