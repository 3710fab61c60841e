cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/late
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_encoder.py tests/test_gpu_rerank_fidelity.py tests/test_gpu_fused_attention.py -x -q --timeout 200 --timeout-method thread > gpurun_out/late/tests.log 2>&1 || exit 1
bash tools/ab_bench.sh late super-rag_amd/super_rag_amd/lib/ab/libsrmi_early.so super-rag_amd/super_rag_amd/lib/ab/libsrmi_late.so > gpurun_out/late/ab.log 2>&1 || exit 1
