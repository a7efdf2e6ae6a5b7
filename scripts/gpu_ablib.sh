# A/B of library builds (build_variants/lib_NAME.so, "default" = the in-tree library),
# processes interleaved over rounds.  usage: gpu_ablib.sh ROUNDS "VARIANT..." NAME...
#   VARIANT = ab.py variant spec (e.g. grid_fast:64:PT_PIPES=16)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$1; V=$2; shift 2
export GPU_MAX_HW_QUEUES=16
for r in $(seq 1 $R); do
  for n in "$@"; do
    if [ "$n" = default ]; then L=$PWD/pathtracerap_amd/libpathtracer_amd.so; else L=$PWD/build_variants/lib_$n.so; fi
    PT_LIB_PATH=$L timeout -k 10 300 python scripts/ab.py --variants $V --rounds 2 --steps 16 > gpurun_out/ablib_$n.json 2> gpurun_out/ablib_$n.err || { tail -5 gpurun_out/ablib_$n.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ablib_$n.json')); print('round $r $n', {k: v['Mrays_s'] for k, v in d.items()})"
  done
done
