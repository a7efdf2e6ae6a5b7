# Traversal statistics of the persistent traces (PT_TRACE_STATS build,
# build_variants/lib_stats.so): wave iterations per segment, lanes per phase.
# usage: gpu_stats.sh [ntri]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PT_LIB_PATH=$PWD/build_variants/lib_stats.so GPU_MAX_HW_QUEUES=16
N=${1:-100000}
timeout -k 10 300 python scripts/ab.py --ntri $N --variants "grid_fast:64:PT_PIPES=16,PT_DEBUG_ABLATE=20" "bvh:64:PT_PIPES=16,PT_DEBUG_ABLATE=16" --rounds 1 --steps 4 > gpurun_out/stats_$N.json 2> gpurun_out/stats_$N.err || { tail -5 gpurun_out/stats_$N.err; exit 1; }
cat gpurun_out/stats_$N.json
