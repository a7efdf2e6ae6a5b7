# A/B: pipelines (iterations in flight) 16 / 20 / 24 / 32, each with one hardware queue per pipeline
# stream, as separate bench.py processes (GPU_MAX_HW_QUEUES is read once per process, so an in-process
# A/B cannot vary it), interleaved rounds; configs[1] and configs[4] (10M, 16 bounces).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
B="--no-cpu-baseline --no-profile --alt-accel= --targets= --no-full-runs --steps 20 --warmup 5"
for r in 1 2; do
  for w in "" "--ntri 10000000 --bounces 16 --inmem"; do
    for p in 16 20 24 32; do
      timeout -k 10 300 python bench.py $B $w --pipelines $p --hw-queues $p > gpurun_out/pipes.json 2> gpurun_out/pipes.err || { tail -5 gpurun_out/pipes.err; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/pipes.json')); print('round $r', '${w:-100k}'[:8], 'pipes $p', d['value'], d['ms_per_step'], d['config']['trace_faults'])" | tee -a gpurun_out/pipes_rounds.txt
    done
  done
done
