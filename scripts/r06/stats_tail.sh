# stats build at the round-6 code: phase iterations / lanes, cycle shares, and the tail launches'
# own cycle split (slots 70..75) at 100k and 10M (where the drain tail is longest)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
PT_LIB_PATH=$PWD/build_variants/lib_stats.so timeout -k 10 600 python -u scripts/ab.py --rounds 1 --steps 8 --variants grid_fast:64:PT_DEBUG_ABLATE=16 grid_fast:64:PT_DEBUG_ABLATE=32 grid_fast:64:PT_DEBUG_ABLATE=2052 > gpurun_out/stats6_100k.json 2> gpurun_out/stats6_100k.err &&
PT_LIB_PATH=$PWD/build_variants/lib_stats.so timeout -k 10 600 python -u scripts/ab.py --inmem --ntri 10000000 --bounces 16 --rounds 1 --steps 8 --variants grid_fast:64:PT_DEBUG_ABLATE=16 grid_fast:64:PT_DEBUG_ABLATE=32 grid_fast:64:PT_DEBUG_ABLATE=2052 > gpurun_out/stats6_10m.json 2> gpurun_out/stats6_10m.err
