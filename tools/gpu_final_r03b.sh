# Round-3 final tree, part 2: rocprofv3 kernel trace + PMC passes of the bench, config 5, fp8 mode 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r03f
bash tools/profile_round.sh r03f || exit 1
python3 tools/pmc_traffic.py gpurun_out/prof_r03f gpurun_out/r03f/r03f_pmc_traffic.json > gpurun_out/r03f/pmc_traffic.log 2>&1 || exit 1
python3 tools/rocprof_vs_bench.py gpurun_out/prof_r03f > gpurun_out/r03f/rocprof_vs_bench.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --workload config5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03f/bench_config5.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --fp8 3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03f/bench_fp8m3.log 2>&1 || exit 1
cp gpurun_out/prof_r03f/trace/run_kernel_stats.csv gpurun_out/r03f/r03f_rocprof_kernel_stats.csv 2>/dev/null
cp gpurun_out/prof_r03f/bench_trace.log gpurun_out/r03f/bench_trace.log 2>/dev/null
# the raw traces / counter CSVs exceed gpurun's 64 MiB copy-back: keep only the summaries
find gpurun_out/prof_r03f -name "*.csv" -size +1M -delete
exit 0
