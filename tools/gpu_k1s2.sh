cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/k1s2
for b in 32 64; do
  SR_SCAN_STREAM=1 timeout -k 10 200 python -u tools/bench_search_fp8.py --batch $b --k 10 --steps 10 > gpurun_out/k1s2/small_b$b.json 2>&1 || exit 1
  SR_SCAN_STREAM=2 timeout -k 10 200 python -u tools/bench_search_fp8.py --batch $b --k 10 --steps 10 > gpurun_out/k1s2/stream_b$b.json 2>&1 || exit 1
done
bash tools/k1_place_probe.sh || exit 1
