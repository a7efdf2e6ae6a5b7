# SQ / TCC counter passes on the bench (separate passes, kernel counters only).  usage: gpu_sqpmc.sh ACCEL
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ACC=${1:-grid_fast}
B="bench.py --accel $ACC --alt-accel= --steps 4 --warmup 1 --no-cpu-baseline --no-profile"
i=0
timeout -k 10 120 rocprofv3 -L > gpurun_out/avail.txt 2>&1 || true
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
         "TCC_HIT_sum TCC_MISS_sum" "SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE" \
         "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C -d gpurun_out/sq${ACC}$i -o run --output-format csv -- python3 $B > gpurun_out/sq$i.log 2>&1 || { tail -5 gpurun_out/sq$i.log; echo "pass $i failed"; }
done
python3 scripts/pmc_table.py gpurun_out/sq${ACC}1 gpurun_out/sq${ACC}2 gpurun_out/sq${ACC}3 gpurun_out/sq${ACC}4
