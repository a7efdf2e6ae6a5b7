#!/bin/bash
# Build the library with csrc/renderer.hip replaced by FILE into build_variants/lib_NAME.so
# (the other sources from the working tree).  usage: build_file.sh NAME FILE [extra -D flags]
set -e
cd "$(dirname "$0")/.."
NAME=$1; FILE=$(realpath "$2"); shift 2
T=$(mktemp -d)
mkdir -p $T/pathtracerap_amd
cp -r pathtracerap_amd/csrc $T/pathtracerap_amd/ && cp -r include $T/
cp "$FILE" $T/pathtracerap_amd/csrc/renderer.hip
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -Wno-unused-result -Wno-unused-value -Wno-pass-failed $*"
mkdir -p build_variants
for s in scene bvh capi; do /opt/rocm/bin/hipcc $F -x hip -c $T/pathtracerap_amd/csrc/$s.cpp -o $T/$s.o & done
/opt/rocm/bin/hipcc $F -c $T/pathtracerap_amd/csrc/renderer.hip -o $T/renderer.o 2>/dev/null
wait
/opt/rocm/bin/hipcc $F -shared -o build_variants/lib_$NAME.so $T/*.o
rm -rf $T
echo built build_variants/lib_$NAME.so from $FILE
