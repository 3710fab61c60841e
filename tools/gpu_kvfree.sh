cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/kvfree
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py -x -q --timeout 200 --timeout-method thread -k "kvfree or bge_reranker or ln_folded or fp8" > gpurun_out/kvfree/tests1.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_rerank_fidelity.py tests/test_gpu_fused_attention.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -k "rerank or fidelity or fused or config3" > gpurun_out/kvfree/tests2.log 2>&1 || exit 1
bash tools/ab_bench.sh kvfree super-rag_amd/super_rag_amd/lib/libsrmi.so@SR_KVFREE_CLS=0 super-rag_amd/super_rag_amd/lib/libsrmi.so@SR_KVFREE_CLS=1 > gpurun_out/kvfree/ab.log 2>&1 || exit 1
