# The start / end ramp of a renderLoop call: the last wave's trace launches sized for latency
# (PT_FINAL_RPL=0: every block of the grid; unset: 4 rays per lane as every iteration) and the tail
# launches' grid (PT_TAIL_BLOCKS 512 vs the default 2048), as separate processes, interleaved rounds:
# renderLoop time at 16 / 20 / 64 iterations (scripts/enqueue_probe.py).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
for r in 1 2; do
  for v in "PT_X=0" "PT_FINAL_RPL=0" "PT_TAIL_BLOCKS=512" "PT_TAIL_BLOCKS=1024"; do
    env $v timeout -k 10 300 python scripts/enqueue_probe.py --steps 16 20 64 > gpurun_out/rp.json || exit 1
    echo "r$r 100k $v $(cat gpurun_out/rp.json)" | tee -a gpurun_out/ab_ramp.txt
    env $v timeout -k 10 300 python scripts/enqueue_probe.py --ntri 10000000 --inmem --bounces 16 --steps 16 20 48 > gpurun_out/rp.json || exit 1
    echo "r$r 10M $v $(cat gpurun_out/rp.json)" | tee -a gpurun_out/ab_ramp.txt
  done
done
