# stats build at the final round-6 code: phase iterations / lanes, cycle shares (main and tail launches),
# certificate outcomes and the fast certificate's failed conditions, at configs[1] and 10M
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
PT_LIB_PATH=$PWD/build_variants/lib_stats.so timeout -k 10 600 python -u scripts/ab.py --rounds 1 --steps 8 --variants grid_fast:64:PT_DEBUG_ABLATE=16 grid_fast:64:PT_DEBUG_ABLATE=32 grid_fast:64:PT_DEBUG_ABLATE=2052 > gpurun_out/stats_final_100k.json 2> gpurun_out/stats_final_100k.err &&
PT_LIB_PATH=$PWD/build_variants/lib_stats.so timeout -k 10 600 python -u scripts/ab.py --inmem --ntri 10000000 --bounces 16 --rounds 1 --steps 8 --variants grid_fast:64:PT_DEBUG_ABLATE=16 grid_fast:64:PT_DEBUG_ABLATE=32 grid_fast:64:PT_DEBUG_ABLATE=2052 > gpurun_out/stats_final_10m.json 2> gpurun_out/stats_final_10m.err
