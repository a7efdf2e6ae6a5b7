# Timing-only ablation of the grid_fast node-pruning growth (stats build): full voxel, half voxel, none.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PT_LIB_PATH=build_variants/lib_stats.so GPU_MAX_HW_QUEUES=16 timeout -k 10 600 python scripts/ab.py --variants grid_fast:64:PT_PIPES=16 grid_fast:64:PT_PIPES=16,PT_DEBUG_ABLATE=512 grid_fast:64:PT_PIPES=16,PT_DEBUG_ABLATE=1024 --rounds 3 --steps 8 > gpurun_out/ab_gablate.json 2> gpurun_out/ab_gablate.err
rc=$?; cat gpurun_out/ab_gablate.json; tail -3 gpurun_out/ab_gablate.err; exit $rc
