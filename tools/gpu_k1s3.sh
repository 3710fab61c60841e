cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/k1s2
timeout -k 10 120 ./tools/diag/gemm4w 131072 10 > gpurun_out/k1s2/gemm4w.log 2>&1 || exit 1
bash tools/gpu_k1s2.sh
