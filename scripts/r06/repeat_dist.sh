# The driver's bench line three times in a row (run-to-run spread at the final code), and the multi-rank
# path rehearsed on the one-GPU box: bench.py --gpus 2 over gloo, two ranks sharing the card (a path
# check -- barriers, the accumulator all-reduce, max-over-ranks timing -- not a scaling number).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/dist &&
for r in 1 2 3; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/rep$r.json 2> gpurun_out/rep$r.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/rep$r.json')); print('run $r', d['value'], d['ms_per_step'], {k: t['value'] for k, t in d['targets'].items()}, d['alt_mode']['value'])" | tee -a gpurun_out/bench_repeat.txt
done &&
timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 > gpurun_out/dist/bench_gloo2_one_gpu.json 2> gpurun_out/dist/bench_gloo2_one_gpu.err &&
cat gpurun_out/dist/bench_gloo2_one_gpu.json
