set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/ab.py --variants bvh:256 bvh:128 bvh:64 grid:256 grid:64 --rounds 3 --steps 8 > gpurun_out/ab.json 2> gpurun_out/ab.err
rc=$?; cat gpurun_out/ab.json; tail -3 gpurun_out/ab.err; exit $rc
