set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_fused_attention.py tests/test_gpu_encoder.py tests/test_gpu_pipeline.py > gpurun_out/perm_tests.log 2>&1 || exit 1
bash tools/ab_bench.sh perm ab/libsrmi_head.so ab/libsrmi_head.so@SR_FUSED_QKV_ATTN=1
