cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/y8
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_encoder.py tests/test_gpu_rerank_fidelity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/y8/tests.log 2>&1 || exit 1
for r in 1 2; do
  for lib in y8old y8line; do
    SUPER_RAG_AMD_LIB=super-rag_amd/super_rag_amd/lib/ab/libsrmi_$lib.so timeout -k 10 240 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-extras --fp8 3 > gpurun_out/y8/${lib}_r$r.log 2>&1 || exit 1
  done
done
