#!/bin/bash
# Round profile on the GPU box (run from the repo root via gpurun):
#   1. kernel-trace + stats of the default bench command
#   2. FETCH_SIZE and WRITE_SIZE in separate PMC passes (MI355X_MICROARCH.md: one TCC counter
#      group per pass) over a 1-step bench
#   3. MFMA busy cycles + GRBM_GUI_ACTIVE (matrix-pipe utilisation and the clock actually held)
# All with --no-extras: the extras (drop-in flow, peaks, B = 32 search) launch the same kernels at
# other shapes, which would mix into the per-launch means of the timed step's kernels.
# Summaries: python tools/pmc_traffic.py gpurun_out/prof_<tag> profiles/<tag>_pmc_traffic.json
# Outputs under gpurun_out/prof_<tag>/.
set -e
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
# the native-source fingerprint the counters belong to (bench.py marks a summary stale without it)
python3 -c "import json, bench; print(json.dumps({'source_sha256': bench.source_fingerprint()}))" \
  > $OUT/provenance.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > $OUT/bench_trace.log 2>&1
timeout -k 10 600 rocprofv3 -i tools/pmc_fetch.txt -d $OUT/fetch -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras > $OUT/bench_fetch.log 2>&1
timeout -k 10 600 rocprofv3 -i tools/pmc_write.txt -d $OUT/write -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras > $OUT/bench_write.log 2>&1
timeout -k 10 600 rocprofv3 -i tools/pmc_mfma.txt -d $OUT/mfma -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras > $OUT/bench_mfma.log 2>&1
# 4. the same trace + three PMC passes over config 5's fp8 path (the line's config5 field: bge-m3
#    embed, fp8 scan, BM25 + rrf, reranker in fp8 mode 3) -> $OUT/c5 (pmc_traffic.py: workloads.config5)
C5="python3 bench.py --workload config5 --fp8 3 --no-cpu-baseline --no-extras"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/c5/trace -o run --output-format csv -- \
  $C5 --steps 3 --warmup 1 > $OUT/c5_bench_trace.log 2>&1
for P in fetch write mfma; do
  timeout -k 10 600 rocprofv3 -i tools/pmc_$P.txt -d $OUT/c5/$P -o run --output-format csv -- \
    $C5 --steps 1 --warmup 1 > $OUT/c5_bench_$P.log 2>&1
done
