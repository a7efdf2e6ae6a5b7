# The last wave of iterations with trace launches sized for latency (PT_FINAL_RPL rays per lane for its
# sparse bounces; unset = 4 as every other iteration): renderLoop time at 16 / 20 / 32 iterations
# (scripts/enqueue_probe.py), separate processes, interleaved rounds.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
for r in 1 2; do
  for v in X 0 1 2; do
    env PT_FINAL_RPL=$v timeout -k 10 300 python scripts/enqueue_probe.py --steps 16 20 32 > gpurun_out/fr.json || exit 1
    echo "r$r 100k PT_FINAL_RPL=$v $(cat gpurun_out/fr.json)" | tee -a gpurun_out/final_rpl.txt
    env PT_FINAL_RPL=$v timeout -k 10 300 python scripts/enqueue_probe.py --ntri 10000000 --inmem --bounces 16 --steps 16 20 32 > gpurun_out/fr.json || exit 1
    echo "r$r 10M PT_FINAL_RPL=$v $(cat gpurun_out/fr.json)" | tee -a gpurun_out/final_rpl.txt
  done
done
