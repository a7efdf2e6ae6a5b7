#!/bin/bash
# Build the library from a git revision's sources into build_variants/lib_NAME.so
# usage: build_prev.sh NAME [REV] [extra -D flags]
set -e
cd "$(dirname "$0")/.."
NAME=$1; REV=${2:-HEAD}; shift; shift || true
T=$(mktemp -d)
git archive $REV pathtracerap_amd/csrc include | tar -x -C $T
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -Wno-unused-result -Wno-unused-value $*"
mkdir -p build_variants
for s in scene bvh capi; do /opt/rocm/bin/hipcc $F -x hip -c $T/pathtracerap_amd/csrc/$s.cpp -o $T/$s.o & done
/opt/rocm/bin/hipcc $F -c $T/pathtracerap_amd/csrc/renderer.hip -o $T/renderer.o 2>/dev/null
wait
/opt/rocm/bin/hipcc $F -shared -o build_variants/lib_$NAME.so $T/*.o
rm -rf $T
echo built build_variants/lib_$NAME.so from $REV
