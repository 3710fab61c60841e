#!/bin/bash
# PMC stall study of GEMM shapes (run from the repo root on the GPU box):
#   bash tools/pmc_study.sh TAG  -> gpurun_out/pmc_TAG/<config>_<pass>/...
# Configs: FFN1 shape (N 3072, K 768) shipped / no-epilogue / stores-only / math-only, FFN2 shape.
TAG=${1:-study}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_SCA TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"
P3="TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUSY_max TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum"
run() {  # name, args
  name=$1; shift
  timeout -k 10 120 python3 $GRAFT_REPO_ROOT/tools/gemm_shape.py "$@" > $OUT/${name}_time.log 2>&1 || return 1
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/${name}_p$i -o run --output-format csv -- \
      python3 $GRAFT_REPO_ROOT/tools/gemm_shape.py "$@" --reps 5 > $OUT/${name}_p$i.log 2>&1 || return 1
  done
}
run ffn1_v5 --variant 5 --epi 1 --N 3072 --K 768 &&
run ffn1_v9 --variant 9 --epi 1 --N 3072 --K 768 &&
run ffn1_v11 --variant 11 --epi 1 --N 3072 --K 768 &&
run ffn1_v10 --variant 10 --epi 1 --N 3072 --K 768 &&
run ffn2_v5 --variant 5 --epi 4 --N 768 --K 3072 &&
run ffn2_v9 --variant 9 --epi 4 --N 768 --K 3072
