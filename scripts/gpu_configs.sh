# The other BASELINE configurations: 1M-tri target, metallic 2800x2240, 10M-tri 16-bounce stress,
# and the literal reference-grid mode on the bench workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { name=$1; shift; timeout -k 10 500 python bench.py --no-cpu-baseline "$@" > gpurun_out/cfg_$name.json 2> gpurun_out/cfg_$name.err || { echo "FAIL $name"; tail -5 gpurun_out/cfg_$name.err; exit 1; }; echo "$name $(python3 -c "import json;d=json.load(open('gpurun_out/cfg_$name.json'));a=d.get('alt_mode') or {};print(d['value'],d['ms_per_step'],'alt',a.get('value'),a.get('ms_per_step'))")"; }
run tri1m --ntri 1000000 --steps 16 --warmup 1
run metal2800 --metallic --width 2800 --height 2240 --bounces 5 --steps 8 --warmup 1
run tri10m --ntri 10000000 --bounces 16 --steps 4 --warmup 1
run grid --accel grid --alt-accel= --steps 4 --warmup 1 --no-profile
