# Kernel-trace timelines of the driver's bench line (configs[1], 20 timed iterations) and of configs[4]'s
# 16 timed iterations, folded by scripts/ramp.py into wall-time slices: trace kernels in flight, iteration
# starts / merges -- how much of a short timed region runs with few iterations in flight.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
B="--no-cpu-baseline --no-profile --alt-accel= --targets= --no-full-runs"
bash scripts/gpu_run.sh "ktrace=$B --steps 20 --warmup 5" "ktrace=$B --ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 5" &&
python3 scripts/ramp.py gpurun_out/s1_ktrace 20 > gpurun_out/ramp_100k.txt && python3 scripts/ramp.py gpurun_out/s2_ktrace 20 > gpurun_out/ramp_10m.txt &&
cat gpurun_out/ramp_100k.txt gpurun_out/ramp_10m.txt
