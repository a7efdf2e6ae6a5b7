# node visits per node step / lane minimum at the 4-wide BLAS, and the 4-wide k_trace_bvh (interleaved library builds)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "tests=bvh or drain_continuation or pipelines_bit or ray_sort or trace_faults or graph_replay" \
  "abbench=3@--steps 20 --warmup 5@default,ns4,ns6,ns12,ml4,ml16" \
  "abbench=3@--accel bvh --steps 20 --warmup 5@default,bvhbin,bvhw4" \
  "abbench=2@--steps 20 --warmup 5 --pipelines 1@default,p1s4,p1s8" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,ns4,ns6,ml4"
