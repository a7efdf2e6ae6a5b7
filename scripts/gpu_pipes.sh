# Pipelines / hardware-queue sweep of the bench line (one process per setting).  usage: gpu_pipes.sh "P:Q ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for pq in $1; do
    P=${pq%:*}; Q=${pq#*:}
    timeout -k 10 200 python bench.py --pipelines $P --hw-queues $Q --steps 32 --warmup 2 --no-cpu-baseline --no-profile --alt-accel= > gpurun_out/pipes_$P_$Q.json 2> gpurun_out/pipes.err || { tail -5 gpurun_out/pipes.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/pipes_$P_$Q.json').read().strip().splitlines()[-1]); print('round $r pipes $P queues $Q', d['value'])"
  done
done
