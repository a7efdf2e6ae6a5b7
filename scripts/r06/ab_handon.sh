# Walk hand-ons (default with several pipelines: the main launch only certifies, the tail walks what both
# certificates declined) vs in-place walks in the main launch (PT_WALK_HANDON=0, variant F | 16), after the
# tail stopped re-running the certificates and the tie rule: separate bench.py processes, interleaved,
# configs[1] at 20 and 64 timed iterations and 10M at 32.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
B="--no-cpu-baseline --no-profile --alt-accel= --targets= --no-full-runs --warmup 5"
run() {   # label, env, args
  env $2 timeout -k 10 300 python bench.py $B $3 > gpurun_out/ho.json 2> gpurun_out/ho.err || { tail -5 gpurun_out/ho.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ho.json')); print('$1', d['value'], d['ms_per_step'], d['config']['trace_faults'])" | tee -a gpurun_out/handon_rounds.txt
}
for r in 1 2 3; do
  for v in 1 0; do
    run "r$r 100k s20 handon=$v" "PT_WALK_HANDON=$v" "--steps 20"
    run "r$r 100k s64 handon=$v" "PT_WALK_HANDON=$v" "--steps 64"
  done
done
for r in 1 2; do
  for v in 1 0; do
    run "r$r 10M s32 handon=$v" "PT_WALK_HANDON=$v" "--ntri 10000000 --bounces 16 --inmem --steps 32"
  done
done
