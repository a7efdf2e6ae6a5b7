# Persistent trace A/B: parity tests, then trace variants (env read at allocateOnGPU).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 400 python scripts/ab.py --variants "$@" --rounds 3 --steps 6 > gpurun_out/split.json 2>gpurun_out/split.err || { tail -5 gpurun_out/split.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/split.json'));[print(k, v['ms_per_spp_median'], v['Mrays_s']) for k,v in d.items()]"
