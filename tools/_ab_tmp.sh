set -o pipefail
mkdir -p gpurun_out/gm
i=0
for g in default 2304:1 2304:3 2304:2,3072:2,768:2 3072:4,768:8 768:1 3072:16,768:16 default; do
  i=$((i+1))
  if [ "$g" = default ]; then unset SR_GEMM_GROUP_M; else export SR_GEMM_GROUP_M=$g; fi
  timeout -k 10 300 python -u tools/gemm_bench.py --variants 5 --rounds 2 --M 1638400 > gpurun_out/gm/run${i}_${g//[:,]/_}.log 2>&1 || { echo "fail $g"; exit 1; }
  echo "done $g"
done
