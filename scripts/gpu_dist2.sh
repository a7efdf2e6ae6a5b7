# Rehearse bench.py's multi-rank path (barriers, all-reduce of the accumulator,
# max-over-ranks timing, rank-0 profile pass) with 2 ranks on the one GPU over gloo.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 8 --warmup 1 --dist-backend gloo --no-cpu-baseline > gpurun_out/dist2.out 2> gpurun_out/dist2.err
rc=$?
# gloo prints its connection banner on stdout: keep only the bench's JSON line
grep '^{' gpurun_out/dist2.out | tail -n 1 > gpurun_out/dist2.json || rc=1
cat gpurun_out/dist2.json; tail -5 gpurun_out/dist2.err; exit $rc
