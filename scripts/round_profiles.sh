# The round's profile set on one MI355X, in two gpurun calls (each fits the 20-minute cap):
#   part 1 -- configs[1] (100k triangles, the bench line), both traces:
#     rocprofv3 --kernel-trace --stats at 16 pipelines and at 1 (the roofline pass),
#     FETCH_SIZE / WRITE_SIZE passes (one pipeline: PMC collection serialises dispatches),
#     SQ_INSTS_VALU / SQ_INSTS_SALU passes at 16 pipelines and at 1,
#     the SQ wave-cycle pass (waits, issue, VALU lanes) at 1 pipeline and at 16
#   part 2 -- the north_star target (1M triangles) and configs[4] (10M triangles, 16
#     bounces, scene built in memory), grid_fast: the same stats / FETCH / WRITE / SQ /
#     wave-cycle passes, so bench.py's targets.*.roofline has its own traffic and issue
#   part 3 -- configs[2] (the README scene, scenes/reference_scene.txt, at 2800x2240 and
#     its RENDER block's 5 bounces; metal / coat / diffuse / emissive models): the same
#     passes under bench.py's target key grid_fast_configs2_2800x2240_b5
# Every pass runs --no-full-runs: the counters are per launch, and the SQ per-iteration
# totals divide by the first-bounce dispatches the pass counted (scripts/pmc_summary.py).
# scripts/pmc_summary.py folds the counters into gpurun_out/pmc_round.json (copy to
# profiles/pmc_latest.json, which bench.py reads) and the stats CSVs go to gpurun_out/round/.
#   usage: bash scripts/round_profiles.sh 1|2|3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
part=${1:-1}
B="--targets= --no-cpu-baseline --alt-accel= --no-profile --no-full-runs"
S="--steps 8 --warmup 1"
CYC="SQ_WAVES,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_THREAD_CYCLES_VALU,SQ_INSTS_VALU"
INS="SQ_INSTS_VALU,SQ_INSTS_SALU"
O=gpurun_out/pmc_round.json
mkdir -p gpurun_out/round
stats() {   # copy step N's kernel stats to gpurun_out/round/kernel_stats_NAME.csv
  f=$(find gpurun_out/s$1_prof -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/round/kernel_stats_$2.csv
}
if [ "$part" = 1 ]; then
  K=grid_fast_100000_1280x1024_b8; KB=bvh_100000_1280x1024_b8
  bash scripts/gpu_run.sh \
    "prof=$B" "prof=$B --pipelines 1" "prof=--accel bvh $B" "prof=--accel bvh $B --pipelines 1" \
    "pmc=$B $S --pipelines 1" "pmc=--accel bvh $B $S --pipelines 1" \
    "counters=$INS@$B $S" "counters=$INS@$B $S --pipelines 1" \
    "counters=$INS@--accel bvh $B $S" "counters=$INS@--accel bvh $B $S --pipelines 1" \
    "counters=$CYC@$B $S --pipelines 1" "counters=$CYC@$B $S" || exit $?
  rm -f $O
  python3 scripts/pmc_summary.py $K gpurun_out/s5_pmc_fetch gpurun_out/s5_pmc_write $O > /dev/null &&
  python3 scripts/pmc_summary.py $KB gpurun_out/s6_pmc_fetch gpurun_out/s6_pmc_write $O > /dev/null &&
  python3 scripts/pmc_summary.py sq $K gpurun_out/s7_counters _sq $O > /dev/null &&
  python3 scripts/pmc_summary.py sq $K gpurun_out/s8_counters _sq_p1 $O > /dev/null &&
  python3 scripts/pmc_summary.py sq $KB gpurun_out/s9_counters _sq $O > /dev/null &&
  python3 scripts/pmc_summary.py sq $KB gpurun_out/s10_counters _sq_p1 $O > /dev/null &&
  python3 scripts/pmc_summary.py cycles $K gpurun_out/s11_counters _cycles_p1 $O > /dev/null &&
  python3 scripts/pmc_summary.py cycles $K gpurun_out/s12_counters _cycles $O > /dev/null || exit 1
  stats 1 grid_fast_16p && stats 2 grid_fast_1p && stats 3 bvh_16p && stats 4 bvh_1p || exit 1
  python3 scripts/pmc_table.py gpurun_out/s11_counters > gpurun_out/round/sq_cycles_p1.txt &&
  python3 scripts/pmc_table.py gpurun_out/s12_counters > gpurun_out/round/sq_cycles_16p.txt || exit 1
  echo "part 1: gpurun_out/round/, $O"
elif [ "$part" = 3 ]; then
  C="$B --scene scenes/reference_scene.txt --width 2800 --height 2240"
  KC=grid_fast_configs2_2800x2240_b5
  bash scripts/gpu_run.sh \
    "prof=$C --steps 16" "prof=$C --steps 16 --pipelines 1" "pmc=$C $S --pipelines 1" \
    "counters=$INS@$C $S --pipelines 1" "counters=$CYC@$C $S --pipelines 1" "counters=$CYC@$C $S" || exit $?
  [ -f $O ] || cp profiles/pmc_latest.json $O
  python3 scripts/pmc_summary.py $KC gpurun_out/s3_pmc_fetch gpurun_out/s3_pmc_write $O > /dev/null &&
  python3 scripts/pmc_summary.py sq $KC gpurun_out/s4_counters _sq_p1 $O > /dev/null &&
  python3 scripts/pmc_summary.py cycles $KC gpurun_out/s5_counters _cycles_p1 $O > /dev/null &&
  python3 scripts/pmc_summary.py cycles $KC gpurun_out/s6_counters _cycles $O > /dev/null || exit 1
  stats 1 grid_fast_configs2_16p && stats 2 grid_fast_configs2_1p || exit 1
  python3 scripts/pmc_table.py gpurun_out/s5_counters > gpurun_out/round/sq_cycles_configs2_p1.txt &&
  python3 scripts/pmc_table.py gpurun_out/s6_counters > gpurun_out/round/sq_cycles_configs2_16p.txt || exit 1
  echo "part 3: gpurun_out/round/, $O"
else
  M="$B --ntri 1000000"; T="$B --ntri 10000000 --bounces 16 --inmem"
  K1=grid_fast_1000000_1280x1024_b8; KT=grid_fast_10000000_1280x1024_b16
  bash scripts/gpu_run.sh \
    "prof=$M --steps 16" "prof=$M --steps 16 --pipelines 1" "prof=$T --steps 16" "prof=$T --steps 16 --pipelines 1" \
    "pmc=$M $S --pipelines 1" "pmc=$T $S --pipelines 1" \
    "counters=$INS@$M $S --pipelines 1" "counters=$INS@$T $S --pipelines 1" \
    "counters=$CYC@$M $S --pipelines 1" "counters=$CYC@$T $S --pipelines 1" "counters=$CYC@$T $S" || exit $?
  [ -f $O ] || cp profiles/pmc_latest.json $O
  python3 scripts/pmc_summary.py $K1 gpurun_out/s5_pmc_fetch gpurun_out/s5_pmc_write $O > /dev/null &&
  python3 scripts/pmc_summary.py $KT gpurun_out/s6_pmc_fetch gpurun_out/s6_pmc_write $O > /dev/null &&
  python3 scripts/pmc_summary.py sq $K1 gpurun_out/s7_counters _sq_p1 $O > /dev/null &&
  python3 scripts/pmc_summary.py sq $KT gpurun_out/s8_counters _sq_p1 $O > /dev/null &&
  python3 scripts/pmc_summary.py cycles $K1 gpurun_out/s9_counters _cycles_p1 $O > /dev/null &&
  python3 scripts/pmc_summary.py cycles $KT gpurun_out/s10_counters _cycles_p1 $O > /dev/null &&
  python3 scripts/pmc_summary.py cycles $KT gpurun_out/s11_counters _cycles $O > /dev/null || exit 1
  stats 1 grid_fast_1m_16p && stats 2 grid_fast_1m_1p && stats 3 grid_fast_10m_16p && stats 4 grid_fast_10m_1p || exit 1
  python3 scripts/pmc_table.py gpurun_out/s9_counters > gpurun_out/round/sq_cycles_1m_p1.txt &&
  python3 scripts/pmc_table.py gpurun_out/s10_counters > gpurun_out/round/sq_cycles_10m_p1.txt &&
  python3 scripts/pmc_table.py gpurun_out/s11_counters > gpurun_out/round/sq_cycles_10m_16p.txt || exit 1
  echo "part 2: gpurun_out/round/, $O"
fi
