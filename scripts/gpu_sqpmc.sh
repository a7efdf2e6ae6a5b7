# SQ / TCC counter passes on the default bench (separate passes, kernel counters only).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-profile"
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
         "TCC_HIT_sum TCC_MISS_sum" "SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C -d gpurun_out/sq$i -o run --output-format csv -- python3 $B > gpurun_out/sq$i.log 2>&1 || { tail -5 gpurun_out/sq$i.log; exit 1; }
done
python3 scripts/pmc_table.py gpurun_out/sq1 gpurun_out/sq2 gpurun_out/sq3
