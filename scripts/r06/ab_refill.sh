# Refill threshold of the persistent main trace (PT_TRACE_REFILL: a wave claims new rays once this many
# lanes are idle; default 32 with several pipelines) at the final code: separate bench.py processes,
# interleaved rounds, configs[1] at 20 and 64 timed iterations and 10M at 32.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
B="--no-cpu-baseline --no-profile --alt-accel= --targets= --no-full-runs --warmup 5"
run() {   # label, env, args
  env $2 timeout -k 10 300 python bench.py $B $3 > gpurun_out/rf.json 2> gpurun_out/rf.err || { tail -5 gpurun_out/rf.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/rf.json')); print('$1', d['value'], d['ms_per_step'], d['config']['trace_faults'])" | tee -a gpurun_out/refill_rounds.txt
}
for r in 1 2; do
  for v in 32 24 40 48; do
    run "r$r 100k s20 refill=$v" "PT_TRACE_REFILL=$v" "--steps 20"
    run "r$r 100k s64 refill=$v" "PT_TRACE_REFILL=$v" "--steps 64"
    run "r$r 10M s32 refill=$v" "PT_TRACE_REFILL=$v" "--ntri 10000000 --bounces 16 --inmem --steps 32"
  done
done
