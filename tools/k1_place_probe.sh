#!/bin/bash
# K1 slow-chunk probe (diagnostic, run from the repo root via gpurun): per-chunk scan durations
# of a 10M x 768, B = 256, k = 100 search with FIXED 1M-row chunks and the epilogue disabled, so
# the rate can be read against the rows' position in the buffer (same work per chunk):
#   plain       the store allocated as in the bench
#   predummy    40 GB allocated (and kept) before the store: other physical pages
#   capacity    a 20M-row buffer for the same 10M rows
#   sched       the default chunk schedule (8 x growth), epilogue disabled
# Summary: python tools/k1_schedule.py gpurun_out/k1s2/k1p_*
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SR_SCAN_DIAG_NOEPI=1
export SR_SCAN_STREAM=0
export SR_SCAN_CHUNK=1048576
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/k1s2/k1p_plain -o run -- \
  python3 tools/k1_dvfs_probe.py > gpurun_out/k1s2/k1p_plain.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/k1s2/k1p_predummy -o run -- \
  python3 tools/k1_dvfs_probe.py --predummy-gb 40 > gpurun_out/k1s2/k1p_predummy.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/k1s2/k1p_capacity -o run -- \
  python3 tools/k1_dvfs_probe.py --capacity 20000000 > gpurun_out/k1s2/k1p_capacity.log 2>&1
unset SR_SCAN_CHUNK
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/k1s2/k1p_sched -o run -- \
  python3 tools/k1_dvfs_probe.py > gpurun_out/k1s2/k1p_sched.log 2>&1
python3 tools/k1_schedule.py gpurun_out/k1s2/k1p_plain gpurun_out/k1s2/k1p_predummy gpurun_out/k1s2/k1p_capacity \
  gpurun_out/k1s2/k1p_sched > gpurun_out/k1s2/k1p_summary.json
