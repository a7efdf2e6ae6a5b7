set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
export PT_LIB_PATH=$PWD/build_variants/lib_stats.so
PT_DEBUG_ABLATE=20 timeout -k 10 300 python scripts/ab.py --variants grid_fast:64 "grid_fast:64:PT_TRACE_SPLIT=1,PT_TRACE_FLAGS=64" --rounds 1 --steps 2 > gpurun_out/gfstats.json 2>gpurun_out/gfstats.err || { tail -5 gpurun_out/gfstats.err; exit 1; }
cat gpurun_out/gfstats.json
