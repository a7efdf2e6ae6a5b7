set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/ab.py --variants ${1:-bvh:64 grid_fast:64} --rounds 3 --steps 8 > gpurun_out/ab.json 2> gpurun_out/ab.err
rc=$?; cat gpurun_out/ab.json; tail -3 gpurun_out/ab.err; [ $rc -eq 0 ] || exit $rc
PT_DEBUG_ABLATE=4 timeout -k 10 300 python scripts/ab.py --variants grid_fast:64 --rounds 1 --steps 4 > gpurun_out/ab_diag.json 2>/dev/null; cat gpurun_out/ab_diag.json
