# grid_fast cost breakdown on the stats build (PT_TRACE_STATS=1): full, no walk (1),
# closest-hit only (2), counters (4); fused and persistent BVH for comparison.
set -o pipefail
cd $GRAFT_REPO_ROOT
PT_LIB_PATH=$PWD/build_variants/lib_stats.so timeout -k 10 300 python scripts/ab.py --rounds 3 --steps 4 --variants \
  grid_fast:64 grid_fast:64:PT_DEBUG_ABLATE=1 grid_fast:64:PT_DEBUG_ABLATE=2 grid_fast:64:PT_DEBUG_ABLATE=4 \
  bvh:64:PT_TRACE_SPLIT=0 bvh:64:PT_TRACE_SPLIT=0,PT_DEBUG_ABLATE=8 bvh:64 > gpurun_out/gfablate.json 2> gpurun_out/gfablate.err
rc=$?; cat gpurun_out/gfablate.json; tail -3 gpurun_out/gfablate.err; exit $rc
