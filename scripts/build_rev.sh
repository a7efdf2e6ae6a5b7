#!/bin/bash
# Build the library as it was at git revision REV into build_variants/lib_NAME.so
# (an A/B baseline for scripts/gpu_run.sh abbench / ablib).  usage: build_rev.sh REV NAME ["-DPT_X=1 ..."]
set -e
cd "$(dirname "$0")/.."
REV=$1; NAME=$2; shift 2
D="$*"
T=build_variants/src_$NAME
rm -rf $T && mkdir -p $T
git archive "$REV" pathtracerap_amd/csrc include | tar -x -C $T
cd $T/pathtracerap_amd && mkdir -p o
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wno-unused-result -Wno-unused-value -Wno-pass-failed $D"
for s in scene bvh capi; do /opt/rocm/bin/hipcc $F -x hip -c csrc/$s.cpp -o o/$s.o & done
/opt/rocm/bin/hipcc $F -c csrc/renderer.hip -o o/renderer.o
wait
/opt/rocm/bin/hipcc $F -shared -o ../../lib_$NAME.so o/*.o
cd ../../.. && rm -rf $T
echo built build_variants/lib_$NAME.so from $REV
