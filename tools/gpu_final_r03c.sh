# Round-3 final tree, part 3: rocprofv3 kernel trace + PMC passes of the bench (timed loop only)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r03f
rm -rf gpurun_out/prof_r03f
bash tools/profile_round.sh r03f || exit 1
python3 tools/pmc_traffic.py gpurun_out/prof_r03f gpurun_out/r03f/r03f_pmc_traffic.json > gpurun_out/r03f/pmc_traffic.log 2>&1 || exit 1
python3 tools/rocprof_vs_bench.py gpurun_out/prof_r03f > gpurun_out/r03f/rocprof_vs_bench.txt 2>&1 || exit 1
cp gpurun_out/prof_r03f/trace/run_kernel_stats.csv gpurun_out/r03f/r03f_rocprof_kernel_stats.csv
cp gpurun_out/prof_r03f/bench_trace.log gpurun_out/r03f/bench_trace.log
find gpurun_out/prof_r03f -name "*.csv" -size +1M -delete
exit 0
