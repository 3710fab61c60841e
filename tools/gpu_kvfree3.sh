cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/kvfree3
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_rerank_fidelity.py tests/test_gpu_fused_attention.py tests/test_gpu_flow.py -x -q --timeout 250 --timeout-method thread > gpurun_out/kvfree3/tests.log 2>&1 || exit 1
bash tools/ab_bench.sh kvfree super-rag_amd/super_rag_amd/lib/libsrmi.so@SR_KVFREE_CLS=0 super-rag_amd/super_rag_amd/lib/libsrmi.so@SR_KVFREE_CLS=1 > gpurun_out/kvfree3/ab.log 2>&1 || exit 1
