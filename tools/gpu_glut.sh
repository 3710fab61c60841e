cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/glut
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_encoder.py tests/test_gpu_rerank_fidelity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/glut/tests.log 2>&1 || exit 1
bash tools/ab_bench.sh glut super-rag_amd/super_rag_amd/lib/ab/libsrmi_as.so super-rag_amd/super_rag_amd/lib/ab/libsrmi_lut.so > gpurun_out/glut/ab.log 2>&1 || exit 1
