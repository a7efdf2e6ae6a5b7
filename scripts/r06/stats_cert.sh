# stats build: the fast walk certificate's first failed condition (slots 80..87) at configs[1], 10M and the
# README scene, beside the certificate outcome counts (PT_DEBUG_ABLATE = 4 | 2048)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
PT_LIB_PATH=$PWD/build_variants/lib_stats.so timeout -k 10 300 python -u scripts/ab.py --rounds 1 --steps 4 --variants grid_fast:64:PT_DEBUG_ABLATE=2052 > gpurun_out/stats_cert_100k.json 2> gpurun_out/stats_cert_100k.err &&
PT_LIB_PATH=$PWD/build_variants/lib_stats.so timeout -k 10 300 python -u scripts/ab.py --inmem --ntri 10000000 --bounces 16 --rounds 1 --steps 4 --variants grid_fast:64:PT_DEBUG_ABLATE=2052 > gpurun_out/stats_cert_10m.json 2> gpurun_out/stats_cert_10m.err &&
PT_LIB_PATH=$PWD/build_variants/lib_stats.so timeout -k 10 300 python -u scripts/ab.py --scene scenes/reference_scene.txt --width 2800 --height 2240 --bounces 5 --rounds 1 --steps 2 --variants grid_fast:64:PT_DEBUG_ABLATE=2052 > gpurun_out/stats_cert_c2.json 2> gpurun_out/stats_cert_c2.err &&
cat gpurun_out/stats_cert_*.json
