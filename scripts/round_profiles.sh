# The round's profile set on one MI355X (one gpurun call), for both traces:
#   - rocprofv3 --kernel-trace --stats of the bench command at its 16 pipelines and at 1
#   - FETCH_SIZE / WRITE_SIZE passes (one pipeline: PMC collection serialises dispatches)
#   - SQ_INSTS_VALU / SQ_INSTS_SALU passes at 16 pipelines and at 1
#   - an SQ wave-cycle pass (waits, issue, VALU lanes), one pipeline
#   - rocprofv3 --kernel-trace --stats of the north_star target (1M triangles) and of
#     configs[4] (10M triangles, 16 bounces, scene built in memory), 16 pipelines
# then scripts/pmc_summary.py folds the counters into gpurun_out/pmc_round.json
# (copy to profiles/pmc_latest.json, which bench.py reads for roofline.traffic and
# issue_roofline) and the stats CSVs to gpurun_out/round/.
#   usage: bash scripts/round_profiles.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
B="--targets= --no-cpu-baseline --alt-accel= --no-profile"
S="--steps 8 --warmup 1"          # counter passes: 9 iterations
bash scripts/gpu_run.sh \
  "prof=$B" "prof=$B --pipelines 1" "prof=--accel bvh $B" "prof=--accel bvh $B --pipelines 1" \
  "pmc=$B $S --pipelines 1" "pmc=--accel bvh $B $S --pipelines 1" \
  "counters=SQ_INSTS_VALU,SQ_INSTS_SALU@$B $S" "counters=SQ_INSTS_VALU,SQ_INSTS_SALU@$B $S --pipelines 1" \
  "counters=SQ_INSTS_VALU,SQ_INSTS_SALU@--accel bvh $B $S" \
  "counters=SQ_INSTS_VALU,SQ_INSTS_SALU@--accel bvh $B $S --pipelines 1" \
  "prof=$B --ntri 1000000 --steps 16" "prof=$B --ntri 10000000 --bounces 16 --inmem --steps 16" || exit $?
O=gpurun_out/pmc_round.json
rm -f $O
python3 scripts/pmc_summary.py grid_fast_100000_1280x1024_b8 gpurun_out/s5_pmc_fetch gpurun_out/s5_pmc_write $O > /dev/null &&
python3 scripts/pmc_summary.py bvh_100000_1280x1024_b8 gpurun_out/s6_pmc_fetch gpurun_out/s6_pmc_write $O > /dev/null &&
python3 scripts/pmc_summary.py sq grid_fast_100000_1280x1024_b8 gpurun_out/s7_counters 9 _sq $O > /dev/null &&
python3 scripts/pmc_summary.py sq grid_fast_100000_1280x1024_b8 gpurun_out/s8_counters 9 _sq_p1 $O > /dev/null &&
python3 scripts/pmc_summary.py sq bvh_100000_1280x1024_b8 gpurun_out/s9_counters 9 _sq $O > /dev/null &&
python3 scripts/pmc_summary.py sq bvh_100000_1280x1024_b8 gpurun_out/s10_counters 9 _sq_p1 $O > /dev/null || exit 1
mkdir -p gpurun_out/round
for s in 1 2 3 4 11 12; do
  f=$(find gpurun_out/s${s}_prof -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/round/kernel_stats_s$s.csv
done
# wave-cycle split of the traces (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES) and
# VALU lane use (THREAD_CYCLES_VALU / ACTIVE_INST_VALU / 64), one pipeline: gpurun_out/s1_counters.txt
bash scripts/gpu_run.sh \
  "counters=SQ_WAVES,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_THREAD_CYCLES_VALU,SQ_INSTS_VALU@$B $S --pipelines 1" || exit $?
python3 scripts/pmc_table.py gpurun_out/s1_counters > gpurun_out/round/sq_cycles_p1.txt || exit 1
echo "profiles: gpurun_out/round/ (s1 grid_fast 16p, s2 grid_fast 1p, s3 bvh 16p, s4 bvh 1p, s11 1M tris, s12 10M tris), $O"
