#!/bin/bash
# VGPR / spill / LDS usage of every kernel of one source file (gfx950):
#   tools/kernel_resources.sh super-rag_amd/csrc/k_gemm.hip [extra hipcc flags]
SRC=${1:?source}; shift
OUT=/tmp/sr_kres_$$.s
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-function \
  -I"$(dirname "$0")/../include" --cuda-device-only -S "$SRC" -o $OUT "$@" 2>/dev/null || exit 1
awk '/^[_a-zA-Z0-9]+:.*; @/{name=$1} /; NumVgprs:/{v=$3} /; ScratchSize:/{sc=$3} /; LDSByteSize|group_segment_fixed_size/{l=$NF}
     /; Occupancy:/{printf "%-95s vgpr=%s scratch=%s occ=%s\n", substr(name,1,95), v, sc, $3}' $OUT | c++filt | sed 's/sr::(anonymous namespace):://'
rm -f $OUT
