# Quick interleaved A/B of renderer variants (scripts/ab.py) at 16 pipelines / 16 queues.
# usage: gpu_abq.sh OUTNAME ROUNDS VARIANT...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=$1; R=$2; shift 2
export GPU_MAX_HW_QUEUES=16
timeout -k 10 500 python scripts/ab.py --variants "$@" --rounds $R --steps 8 > gpurun_out/$OUT.json 2> gpurun_out/$OUT.err || { tail -5 gpurun_out/$OUT.err; exit 1; }
cat gpurun_out/$OUT.json
