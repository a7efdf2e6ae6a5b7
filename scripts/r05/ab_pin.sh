# 4-wide node base pointer pinned in SGPRs (no per-visit kernel-argument reload; default) vs HEAD (prev)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "tests=configs1 or window_bitexact or walk_handon or bvh_mode or configs0" \
  "abbench=3@--steps 20 --warmup 5@default,prev" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,prev" \
  "abbench=2@--accel bvh --steps 20 --warmup 5@default,prev"
