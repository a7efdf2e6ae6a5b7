# BLAS leaf-size sweep: timing (no counters) then traversal statistics (PT_DEBUG_ABLATE=8).
# usage: gpu_leaf.sh NTRI LEAF...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
N=$1; shift
for L in "$@"; do
  PT_BVH_LEAF=$L timeout -k 10 300 python scripts/ab.py --ntri $N --variants bvh:64 grid_fast:64 --rounds 3 --steps 6 > gpurun_out/leaf_${N}_$L.json 2>gpurun_out/leaf_$L.err || { tail -5 gpurun_out/leaf_$L.err; exit 1; }
  PT_BVH_LEAF=$L PT_DEBUG_ABLATE=8 timeout -k 10 300 python scripts/ab.py --ntri $N --variants bvh:64 --rounds 1 --steps 2 > gpurun_out/leafst_${N}_$L.json 2>gpurun_out/leafst_$L.err || { tail -5 gpurun_out/leafst_$L.err; exit 1; }
  echo "ntri=$N leaf=$L $(python3 -c "import json;print(json.dumps(json.load(open('gpurun_out/leaf_${N}_$L.json'))), json.dumps(json.load(open('gpurun_out/leafst_${N}_$L.json'))))")"
done
