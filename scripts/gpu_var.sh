# A/B of library variants in build_variants/ (VARIANTS env: ab.py variant specs)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python scripts/ab.py --rounds 3 --steps 4 --variants ${VARIANTS:-grid_fast:64} > gpurun_out/ab_default.json 2>/dev/null || exit 1
echo "default $(tr -d '\n ' < gpurun_out/ab_default.json)"
for L in ${LIBS:-w5}; do
  PT_LIB_PATH=$PWD/build_variants/lib_$L.so timeout -k 10 200 python scripts/ab.py --variants ${VARIANTS:-grid_fast:64} --rounds 3 --steps 4 > gpurun_out/ab_$L.json 2>/dev/null || exit 1
  echo "$L $(tr -d '\n ' < gpurun_out/ab_$L.json)"
done
