#!/bin/bash
# build_variant.sh NAME SRC_HIP: libmlffpcg.so with csrc/kernels_sym.hip replaced by SRC_HIP
# (kernel A/B experiments; load with MLFF_LIB=mlff-preconditioner_amd/lib/variants/NAME.so)
set -eu
NAME=$1; SRC=$2
R=/root/repo/mlff-preconditioner_amd
mkdir -p $R/lib/variants /tmp/variant_$NAME
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -I/root/repo/include -I$R/csrc -c $SRC -o /tmp/variant_$NAME/kernels_sym.o
objs=$(ls $R/build/obj/*.o | grep -v kernels_sym.o)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib $objs /tmp/variant_$NAME/kernels_sym.o -o $R/lib/variants/$NAME.so
echo built $R/lib/variants/$NAME.so
