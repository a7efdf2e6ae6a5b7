# Instruction-cache counters of the trace kernels on the bench (one --pmc pass per accel).  usage: gpu_icache.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for ACC in grid_fast bvh; do
  B="bench.py --accel $ACC --alt-accel= --steps 4 --warmup 1 --no-cpu-baseline --no-profile"
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d gpurun_out/ic_$ACC -o run --output-format csv -- python3 $B > gpurun_out/ic_$ACC.log 2>&1 || { tail -5 gpurun_out/ic_$ACC.log; exit 1; }
  python3 scripts/pmc_table.py gpurun_out/ic_$ACC
done
