# stats build (tail cycle split) at 100k and 10M, then depth-first node order re-measured with more rounds
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
bash scripts/r06/stats_tail.sh &&
bash scripts/gpu_run.sh "tests=bvh4 or iteration_4095 or configs1_last" \
  "ab=--rounds 5 --steps 20 --variants grid_fast:64 grid_fast:64:PT_BVH4_ORDER=1 bvh:64 bvh:64:PT_BVH4_ORDER=1" \
  "ab=--inmem --ntri 10000000 --bounces 16 --rounds 3 --steps 16 --variants grid_fast:64 grid_fast:64:PT_BVH4_ORDER=1"
