#!/bin/bash
# Multi-rank rehearsal on the one-GPU box (final tree): 2 ranks share cuda:0 over gloo
# (SR_BENCH_BACKEND=gloo), the same bench code path the driver's N > 1 run takes over RCCL.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/rehearsal
export SR_BENCH_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-extras \
  > gpurun_out/rehearsal/bench_2rank.log 2>&1 || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29512 bench.py --gpus 2 --workload config5 --steps 3 --warmup 1 --no-cpu-baseline --no-extras \
  > gpurun_out/rehearsal/bench_config5_2rank.log 2>&1 || exit 1
