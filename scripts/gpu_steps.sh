# Bench line at the driver's step count (20) for several pipeline counts, and at 32 / 64 steps.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "20 16" "20 10" "20 20" "32 16" "64 16" "20 16"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps $1 --warmup 5 --pipelines $2 --no-cpu-baseline --no-profile --alt-accel= > gpurun_out/steps_$1_$2.json 2> gpurun_out/steps.err || { tail -5 gpurun_out/steps.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/steps_$1_$2.json')); print('steps $1 pipes $2', d['value'], d['ms_per_step'])"
done
