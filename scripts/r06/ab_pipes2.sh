# Pipelines 16 vs 20 (one hardware queue each) in steady state -- long timed regions, so the ramp at the
# start and end of renderLoop (fewer iterations in flight) weighs little -- and rays per lane 4 vs 8 for
# the large BLAS, both as separate bench.py processes (no in-process order effects), interleaved rounds.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
B="--no-cpu-baseline --no-profile --alt-accel= --targets= --no-full-runs --warmup 5"
run() {   # label, env, args
  env $2 timeout -k 10 300 python bench.py $B $3 > gpurun_out/p2.json 2> gpurun_out/p2.err || { tail -5 gpurun_out/p2.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/p2.json')); print('$1', d['value'], d['ms_per_step'], d['config']['trace_faults'])" | tee -a gpurun_out/pipes2_rounds.txt
}
T10="--ntri 10000000 --bounces 16 --inmem"
for r in 1 2; do
  run "r$r 100k s128 p16" "PT_X=0" "--steps 128 --pipelines 16 --hw-queues 16"
  run "r$r 100k s128 p20" "PT_X=0" "--steps 128 --pipelines 20 --hw-queues 20"
  run "r$r 10M s64 p16" "PT_X=0" "$T10 --steps 64 --pipelines 16 --hw-queues 16"
  run "r$r 10M s64 p20" "PT_X=0" "$T10 --steps 64 --pipelines 20 --hw-queues 20"
  run "r$r 10M s64 p16 rpl4" "PT_TRACE_RPL=4" "$T10 --steps 64 --pipelines 16 --hw-queues 16"
  run "r$r 1M s96 p16" "PT_X=0" "--ntri 1000000 --steps 96 --pipelines 16 --hw-queues 16"
  run "r$r 1M s96 p20" "PT_X=0" "--ntri 1000000 --steps 96 --pipelines 20 --hw-queues 20"
  run "r$r 1M s96 p16 rpl4" "PT_TRACE_RPL=4" "--ntri 1000000 --steps 96 --pipelines 16 --hw-queues 16"
done
