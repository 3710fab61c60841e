# K1 "last chunk is faster" probe: fixed threshold chunks of 3.3M / 2.1M rows (epilogue off), then
# the default schedule with the epilogue on; per-chunk kernel durations from rocprofv3 traces.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/k1p2
export SR_SCAN_STREAM=0
for c in 3300000 2097152; do
  SR_SCAN_DIAG_NOEPI=1 SR_SCAN_CHUNK=$c timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/k1p2/c$c -o run -- \
    python3 tools/k1_dvfs_probe.py > gpurun_out/k1p2/c$c.log 2>&1 || exit 1
done
python3 tools/k1_schedule.py gpurun_out/k1p2/c3300000 gpurun_out/k1p2/c2097152 > gpurun_out/k1p2/summary.json
