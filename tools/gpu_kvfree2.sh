cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/kvfree2
for kv in 0 1; do
  SR_KVFREE_CLS=$kv timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_rerank_fidelity.py -q -s --timeout 250 --timeout-method thread -k "config3 or fidelity" > gpurun_out/kvfree2/kv$kv.log 2>&1
done
exit 0
