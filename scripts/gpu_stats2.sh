# Traversal statistics (stats build) for a list of ab.py variants.
# usage: gpu_stats2.sh OUT VARIANT...   (needs build_variants/lib_stats.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=$1; shift
export PT_LIB_PATH=$PWD/build_variants/lib_stats.so GPU_MAX_HW_QUEUES=16
timeout -k 10 300 python scripts/ab.py --variants "$@" --rounds 1 --steps 4 > gpurun_out/$OUT.json 2> gpurun_out/$OUT.err || { tail -5 gpurun_out/$OUT.err; exit 1; }
python3 - gpurun_out/$OUT.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    print(k, v["Mrays_s"], "iters/seg", v.get("wave_iters_per_segment"), "phase", v.get("phase_iters_per_segment"),
          "lanes", v.get("lanes_per_phase_iter"), "busy", v.get("busy_lanes_per_iter"),
          "drain", v.get("drain_iter_share"), v.get("busy_lanes_per_drain_iter"))
PY
