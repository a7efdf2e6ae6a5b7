set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python scripts/ab.py --rounds 3 --steps 4 --variants grid_fast:64 grid_fast:64:PT_GF_FLAGS=13 \
  grid_fast:64:PT_GF_FLAGS=13,PT_TRACE_REFILL=16 grid_fast:64:PT_GF_FLAGS=13,PT_TRACE_REFILL=48 grid_fast:64:PT_TRACE_REFILL=16 > gpurun_out/ab.json 2>/dev/null || exit 1
tr -d '\n ' < gpurun_out/ab.json; echo
