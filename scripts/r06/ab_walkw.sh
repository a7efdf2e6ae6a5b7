# Walk phase weight (PT_WALK_W; default 8: the walk phase runs when its lanes outnumber the largest other
# phase's x W/4) re-swept after the tie rule made the walk phase cheaper (the full certificate runs in
# about half as many walk iterations).  Library builds, separate processes, interleaved.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
bash scripts/gpu_run.sh "ablib=3@grid_fast:64@default,walkw5,walkw12,walkw16" \
  "ablib=2@grid_fast:64 --ntri 10000000 --inmem --bounces 16@default,walkw5,walkw12,walkw16"
