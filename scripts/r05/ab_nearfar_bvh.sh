# near / far planes in both traces (default) vs the commit before (prev): bvh parity, then A/B
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "tests=bvh or pipelines_bit or ray_sort or drain_continuation or configs1" \
  "abbench=3@--accel bvh --steps 20 --warmup 5@default,prev" \
  "abbench=2@--steps 20 --warmup 5@default,prev"
