#!/bin/bash
# single-read cls_attn_fold: parity tests, then a same-box A/B of the bench (1READ vs two-pass)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/cls1
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py -k "kvfree" -x -v --timeout 120 --timeout-method thread > gpurun_out/cls1/tests.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/cls1/new_$rep.log 2>&1 || exit 1
  SR_CLS_FOLD_1READ=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/cls1/old_$rep.log 2>&1 || exit 1
done
