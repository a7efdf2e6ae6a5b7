# stats build: 4-wide node visits, hit children, pushes, spilled pushes, triangle tests (100k, 1M, 10M)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
PT_LIB_PATH=$PWD/build_variants/lib_stats.so timeout -k 10 600 python -u scripts/ab.py --rounds 1 --steps 8 --variants grid_fast:64:PT_DEBUG_ABLATE=16 > gpurun_out/st_n4_100k.json 2> gpurun_out/st_n4_100k.err &&
PT_LIB_PATH=$PWD/build_variants/lib_stats.so timeout -k 10 600 python -u scripts/ab.py --ntri 1000000 --rounds 1 --steps 8 --variants grid_fast:64:PT_DEBUG_ABLATE=16 > gpurun_out/st_n4_1m.json 2> gpurun_out/st_n4_1m.err &&
PT_LIB_PATH=$PWD/build_variants/lib_stats.so timeout -k 10 600 python -u scripts/ab.py --inmem --ntri 10000000 --bounces 16 --rounds 1 --steps 8 --variants grid_fast:64:PT_DEBUG_ABLATE=16 > gpurun_out/st_n4_10m.json 2> gpurun_out/st_n4_10m.err
