#!/bin/bash
# Variant libraries for same-box A/Bs: k_gemm.hip (or $SRC) rebuilt with extra -D flags, linked with
# the current product / diagnostic objects of the other sources.
#   tools/build_variant.sh NAME "-DFOO=1 -DBAR=0"  -> super-rag_amd/super_rag_amd/lib_ab/libsrmi_NAME.so
#                                                     and libsrmi_diag_NAME.so
set -e
NAME=$1; DEFS=$2; SRC=${SRC:-k_gemm.hip}
cd "$(dirname "$0")/../super-rag_amd"
make -j8 >/dev/null
mkdir -p build_ab super_rag_amd/lib_ab
F="-x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fvisibility=hidden -I../include"
/opt/rocm/bin/hipcc $F $DEFS -c csrc/$SRC -o build_ab/${NAME}.o &
/opt/rocm/bin/hipcc $F -DSR_WITH_DIAG=1 $DEFS -c csrc/$SRC -o build_ab/${NAME}_diag.o &
wait
P=$(ls build/*.o | grep -v "/$SRC.o")
D=$(ls build_diag/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o super_rag_amd/lib_ab/libsrmi_${NAME}.so $P build_ab/${NAME}.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o super_rag_amd/lib_ab/libsrmi_diag_${NAME}.so $D build_ab/${NAME}_diag.o
echo built lib_ab/libsrmi_${NAME}.so lib_ab/libsrmi_diag_${NAME}.so
