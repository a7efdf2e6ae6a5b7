# Time library variants (build_variants/lib_*.so) on the same box, 2 passes interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
for pass in 1 2; do
for L in build_variants/lib_*.so; do
  PT_LIB_PATH=$PWD/$L timeout -k 10 300 python scripts/ab.py --variants ${VARIANTS:-bvh:64 grid_fast:64} --rounds 2 --steps 8 > gpurun_out/var.json 2>/dev/null || { echo "fail $L"; exit 1; }
  echo "$pass $L $(python3 -c "import json;d=json.load(open('gpurun_out/var.json'));print(' '.join(f'{k}={v[\"ms_per_spp_median\"]}' for k,v in d.items()))")"
done
done
