#!/bin/bash
# Interleaved A/B of runtime environment settings on the bench workload, one
# process per run (settings read once per process, e.g. PT_BVH_LEAF, take effect).
#   usage: bash scripts/envsweep.sh ROUNDS "BENCH ARGS" "ENV1" "ENV2" ...   (ENV: "" or "A=1 B=2")
# prints: round, settings, Mrays/s, ms per step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rounds=$1; bargs=$2; shift 2
for r in $(seq 1 "$rounds"); do
  k=0
  for e in "$@"; do
    k=$((k + 1))
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --alt-accel= --targets= --no-full-runs $bargs \
      > gpurun_out/envsweep_$k.json 2> gpurun_out/envsweep_$k.err || { tail -5 gpurun_out/envsweep_$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/envsweep_$k.json')); print('round $r [${e:-default}]', d['value'], d['ms_per_step'], 'faults', d['config']['trace_faults'])"
  done
done
