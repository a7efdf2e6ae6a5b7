# Host enqueue time of a renderLoop call vs its GPU time (scripts/enqueue_probe.py), default launches and
# hipGraph replay (PT_GRAPH=1), 100k and 10M; separate processes.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
timeout -k 10 300 python scripts/enqueue_probe.py --steps 16 20 32 64 128 > gpurun_out/enq_100k.json &&
PT_GRAPH=1 timeout -k 10 300 python scripts/enqueue_probe.py --steps 16 20 32 64 128 > gpurun_out/enq_100k_graph.json &&
timeout -k 10 300 python scripts/enqueue_probe.py --ntri 10000000 --inmem --bounces 16 --steps 16 20 32 64 > gpurun_out/enq_10m.json &&
PT_GRAPH=1 timeout -k 10 300 python scripts/enqueue_probe.py --ntri 10000000 --inmem --bounces 16 --steps 16 20 32 64 > gpurun_out/enq_10m_graph.json &&
cat gpurun_out/enq_*.json
