# rocprofv3 kernel trace (timestamps) of a bench run, for timeline analysis
# (scripts/timeline.py).  usage: gpu_ktrace.sh ACCEL [extra bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ACC=${1:-grid_fast}; shift
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt_$ACC -o run --output-format csv -- python3 bench.py --accel $ACC --alt-accel= --steps 16 --warmup 2 --no-cpu-baseline --no-profile "$@" > gpurun_out/kt_$ACC.log 2>&1 || { tail -20 gpurun_out/kt_$ACC.log; exit 1; }
tail -1 gpurun_out/kt_$ACC.log
python3 scripts/timeline.py gpurun_out/kt_$ACC
