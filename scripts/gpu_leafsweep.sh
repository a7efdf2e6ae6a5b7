# BLAS leaf-size sweep at 16 pipelines (PT_BVH_LEAF read at scene build), two passes interleaved.
# usage: gpu_leafsweep.sh LEAF...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=16
for pass in 1 2; do
  for L in "$@"; do
    PT_BVH_LEAF=$L timeout -k 10 300 python scripts/ab.py --variants grid_fast:64:PT_PIPES=16 bvh:64:PT_PIPES=16 --rounds 2 --steps 16 > gpurun_out/leaf_$L.json 2> gpurun_out/leaf_$L.err || { tail -5 gpurun_out/leaf_$L.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/leaf_$L.json')); print('pass $pass leaf $L', {k: v['Mrays_s'] for k, v in d.items()})"
  done
done
