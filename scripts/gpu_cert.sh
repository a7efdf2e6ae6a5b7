set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python scripts/ab.py --rounds 3 --steps 4 --variants grid_fast:64 grid_fast:64:PT_GF_SPLIT=0 > gpurun_out/ab.json 2>/dev/null || exit 1
echo "default $(tr -d '\n ' < gpurun_out/ab.json)"
PT_LIB_PATH=$PWD/build_variants/lib_nocert.so timeout -k 10 300 python scripts/ab.py --rounds 3 --steps 4 --variants grid_fast:64 grid_fast:64:PT_GF_SPLIT=0 > gpurun_out/ab_nc.json 2>/dev/null || exit 1
echo "nocert $(tr -d '\n ' < gpurun_out/ab_nc.json)"
PT_LIB_PATH=$PWD/build_variants/lib_stats.so timeout -k 10 300 python scripts/ab.py --rounds 1 --steps 4 --variants grid_fast:64:PT_DEBUG_ABLATE=32 grid_fast:64:PT_DEBUG_ABLATE=4 > gpurun_out/ab_gfst.json 2>/dev/null || exit 1
tr -d '\n ' < gpurun_out/ab_gfst.json; echo
