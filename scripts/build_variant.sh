#!/bin/bash
# Build a variant of the library with extra -D flags into build_variants/lib_NAME.so
# (timed with PT_LIB_PATH=...; see scripts/gpu_variants.sh).  usage: build_variant.sh NAME "-DPT_X=1 ..."
set -e
cd "$(dirname "$0")/../pathtracerap_amd"
NAME=$1; shift
D="$*"
OUT=../build_variants/obj_$NAME
mkdir -p $OUT
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wno-unused-result -Wno-unused-value -Wno-pass-failed $D"
for s in scene bvh capi; do /opt/rocm/bin/hipcc $F -x hip -c csrc/$s.cpp -o $OUT/$s.o & done
/opt/rocm/bin/hipcc $F -c csrc/renderer.hip -o $OUT/renderer.o
wait
/opt/rocm/bin/hipcc $F -shared -o ../build_variants/lib_$NAME.so $OUT/*.o
echo built build_variants/lib_$NAME.so
