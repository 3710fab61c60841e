set -o pipefail
bash tools/ab_bench.sh stagger ab/libsrmi_head.so ab/libsrmi_head.so@SR_GEMM_STAGGER=2 ab/libsrmi_head.so@SR_GEMM_STAGGER=4 ab/libsrmi_head.so@SR_GEMM_STAGGER=8
