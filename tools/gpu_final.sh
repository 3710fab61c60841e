#!/bin/bash
# Final-tree evidence, tag $1 (e.g. r03g), part $2:
#   1  the driver's own commands: GPU tests, smoke, default bench 20 / 5
#   2  rocprofv3 kernel trace + PMC passes of the bench (tools/profile_round.sh), config 5, fp8 modes
#      3 / 4, the bench with bge-reranker-v2-m3 (24 layers) as the reranker
TAG=${1:?tag}; PART=${2:?part}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG
if [ "$PART" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 > gpurun_out/$TAG/gpu_tests.log 2>&1 || exit 1
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit 1
  timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/$TAG/bench_20x5.log 2>&1 || exit 1
else
  rm -rf gpurun_out/prof_$TAG
  bash tools/profile_round.sh $TAG || exit 1
  python3 tools/pmc_traffic.py gpurun_out/prof_$TAG gpurun_out/$TAG/${TAG}_pmc_traffic.json > gpurun_out/$TAG/pmc_traffic.log 2>&1 || exit 1
  python3 tools/rocprof_vs_bench.py gpurun_out/prof_$TAG > gpurun_out/$TAG/rocprof_vs_bench.txt 2>&1 || exit 1
  cp gpurun_out/prof_$TAG/trace/run_kernel_stats.csv gpurun_out/$TAG/${TAG}_rocprof_kernel_stats.csv
  cp gpurun_out/prof_$TAG/bench_trace.log gpurun_out/$TAG/bench_trace.log
  # the raw traces / counter CSVs exceed gpurun's 64 MiB copy-back: keep only the summaries
  find gpurun_out/prof_$TAG -name "*.csv" -size +1M -delete
  timeout -k 10 400 python -u bench.py --workload config5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/$TAG/bench_config5.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --fp8 3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/$TAG/bench_fp8m3.log 2>&1 || exit 1
  timeout -k 10 400 python -u bench.py --rerank-model bge-reranker-v2-m3 --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/$TAG/bench_v2m3.log 2>&1 || exit 1
fi
exit 0
