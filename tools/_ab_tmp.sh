set -o pipefail
mkdir -p gpurun_out/rp
for r in 1 2; do
for v in rp nopf; do
SUPER_RAG_AMD_LIB=ab/libsrmi_$v.so timeout -k 10 300 python -u tools/gemm_bench.py --variants 5 --rounds 2 --M 1638400 --no-parity > gpurun_out/rp/gemm_${v}_$r.log 2>&1 || exit 1
done; done
bash tools/ab_bench.sh rp ab/libsrmi_rp.so ab/libsrmi_nopf.so
