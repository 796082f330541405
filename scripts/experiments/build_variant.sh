#!/bin/bash
# build_variant.sh NAME SRC_HIP [UNIT]: libmlffpcg.so with csrc/UNIT.hip (default
# kernels_sym) replaced by SRC_HIP (kernel A/B experiments; load the result with
# MLFF_LIB=mlff-preconditioner_amd/lib/variants/NAME.so)
set -eu
NAME=$1; SRC=$2; UNIT=${3:-kernels_sym}
R=/root/repo/mlff-preconditioner_amd
mkdir -p $R/lib/variants /tmp/variant_$NAME
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -I/root/repo/include -I$R/csrc -c $SRC -o /tmp/variant_$NAME/$UNIT.o
objs=$(ls $R/build/obj/*.o | grep -v "/$UNIT.o")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib $objs /tmp/variant_$NAME/$UNIT.o -o $R/lib/variants/$NAME.so
echo built $R/lib/variants/$NAME.so
