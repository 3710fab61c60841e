cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/s512
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py -x -q --timeout 250 --timeout-method thread -k "kvfree" > gpurun_out/s512/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --pair-len 512 --passage-len 478 --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/s512/bench_pair512.log 2>&1 || exit 1
SR_KVFREE_CLS=0 timeout -k 10 400 python -u bench.py --pair-len 512 --passage-len 478 --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/s512/bench_pair512_kv.log 2>&1 || exit 1
