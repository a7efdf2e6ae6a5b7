# GRID_FAST overflow pool check: GPU tests, tier counters at 100k / 1M tris, then the BASELINE configs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for N in 100000 1000000; do
  PT_DEBUG_ABLATE=4 timeout -k 10 300 python scripts/ab.py --variants grid_fast:64 bvh:64 --rounds 2 --steps 4 --ntri $N > gpurun_out/diag_$N.json 2>gpurun_out/diag_$N.err || { tail -5 gpurun_out/diag_$N.err; exit 1; }
  echo "ntri=$N $(python3 -c "import json;print(json.dumps(json.load(open('gpurun_out/diag_$N.json'))))")"
done
bash scripts/gpu_configs.sh
