# persistent grid_fast trace: GPU suite, then in-process A/B of the variants.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python scripts/ab.py --rounds 3 --steps 4 --variants grid_fast:64 grid_fast:64:PT_GF_SPLIT=0 \
  grid_fast:64:PT_GF_FLAGS=8 grid_fast:64:PT_TRACE_REFILL=16 grid_fast:64:PT_TRACE_REFILL=48 \
  grid_fast:64:PT_TRACE_WAVES_PER_CU=16 grid_fast:64:PT_TRACE_WAVES_PER_CU=32 > gpurun_out/ab_gf.json 2> gpurun_out/ab_gf.err
rc=$?; cat gpurun_out/ab_gf.json; tail -3 gpurun_out/ab_gf.err; exit $rc
