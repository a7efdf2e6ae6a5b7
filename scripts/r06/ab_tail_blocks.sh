# k_trace_gf's tail launches on a smaller grid (PT_TAIL_BLOCKS; default the main launch's 2048 = 8 waves
# per CU): blocks past the records exit at once, but each still needs a wave slot and its 9 KB of LDS to
# start, so on a GPU full of other pipelines' traces the launch lasts until all 2048 got one.  Separate
# bench.py processes, interleaved; 20 timed iterations (the driver's line) and steady state.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
B="--no-cpu-baseline --no-profile --alt-accel= --targets= --no-full-runs --warmup 5"
run() {   # label, env, args
  env $2 timeout -k 10 300 python bench.py $B $3 > gpurun_out/tb.json 2> gpurun_out/tb.err || { tail -5 gpurun_out/tb.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/tb.json')); print('$1', d['value'], d['ms_per_step'], d['config']['trace_faults'])" | tee -a gpurun_out/tail_blocks_rounds.txt
}
T10="--ntri 10000000 --bounces 16 --inmem"
for r in 1 2; do
  for v in 2048 1024 512; do
    run "r$r 100k s20 tb$v" "PT_TAIL_BLOCKS=$v" "--steps 20"
    run "r$r 100k s96 tb$v" "PT_TAIL_BLOCKS=$v" "--steps 96"
    run "r$r 10M s48 tb$v" "PT_TAIL_BLOCKS=$v" "$T10 --steps 48"
  done
done
