# Memory-pipeline counters of k_trace_gf, one pipeline (100k configs[1] and 10M configs[4]):
# L1->L2 read latency, L2 hit rate, L1 TLB misses, TA/TD busy, VMEM/LDS instruction counts
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
B="--targets= --no-cpu-baseline --alt-accel= --no-profile --no-full-runs --steps 4 --warmup 1 --pipelines 1"
C1="TA_BUSY_avr TD_TD_BUSY_sum GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $C1 -d gpurun_out/mem100k -o run --output-format csv -- python3 bench.py $B > gpurun_out/mem100k.log 2>&1 &&
python3 scripts/pmc_table.py gpurun_out/mem100k > gpurun_out/mem100k.txt &&
timeout -s KILL 180 rocprofv3 --pmc $C1 -d gpurun_out/mem10m -o run --output-format csv -- python3 bench.py $B --ntri 10000000 --bounces 16 --inmem > gpurun_out/mem10m.log 2>&1 &&
python3 scripts/pmc_table.py gpurun_out/mem10m > gpurun_out/mem10m.txt &&
C2="TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C2 -d gpurun_out/mem100k_b -o run --output-format csv -- python3 bench.py $B > gpurun_out/mem100k_b.log 2>&1 &&
python3 scripts/pmc_table.py gpurun_out/mem100k_b > gpurun_out/mem100k_b.txt
