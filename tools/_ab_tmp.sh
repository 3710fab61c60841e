set -o pipefail
mkdir -p gpurun_out/qa
for v in 0 1 2; do
  SR_QA_DIAG=$v timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/qa/diag$v.log 2>&1 || { echo "fail $v"; exit 1; }
done
SR_FUSED_QKV_ATTN=0 timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/qa/unfused.log 2>&1
