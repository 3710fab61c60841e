cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/kvfree6
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py -x -q --timeout 200 --timeout-method thread -k "kvfree or bge_reranker" > gpurun_out/kvfree6/tests.log 2>&1 || exit 1
bash tools/ab_bench.sh kvfree6 super-rag_amd/super_rag_amd/lib/libsrmi.so@SR_KVFREE_CLS=0 super-rag_amd/super_rag_amd/lib/libsrmi.so@SR_KVFREE_CLS=1 > gpurun_out/kvfree6/ab.log 2>&1 || exit 1
