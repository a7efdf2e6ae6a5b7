# Persistent trace A/B: parity tests for BVH, then fused vs split with refill thresholds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 400 python scripts/ab.py --variants bvh:64:PT_TRACE_SPLIT=0 bvh:64 bvh:64:PT_TRACE_REFILL=4 bvh:64:PT_TRACE_REFILL=32 bvh:64:PT_TRACE_REFILL=48 bvh:64:PT_TRACE_WAVES_PER_CU=12 --rounds 3 --steps 6 > gpurun_out/split.json 2>gpurun_out/split.err || { tail -5 gpurun_out/split.err; exit 1; }
cat gpurun_out/split.json
