set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python scripts/ab.py --rounds 3 --steps 4 --variants grid_fast:64 grid_fast:64:PT_GF_FLAGS=0 grid_fast:64:PT_GF_FLAGS=1 > gpurun_out/ab_gf.json 2> gpurun_out/ab_gf.err || exit 1
cat gpurun_out/ab_gf.json
PT_LIB_PATH=$PWD/build_variants/lib_stats.so timeout -k 10 300 python scripts/ab.py --rounds 1 --steps 4 --variants grid_fast:64:PT_DEBUG_ABLATE=16 grid_fast:64:PT_DEBUG_ABLATE=16,PT_GF_FLAGS=1 bvh:64:PT_DEBUG_ABLATE=16 > gpurun_out/ab_gfst.json 2> gpurun_out/ab_gfst.err
rc=$?; cat gpurun_out/ab_gfst.json; tail -3 gpurun_out/ab_gfst.err; exit $rc
