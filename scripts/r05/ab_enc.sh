# pre-encoded leaf links in Bvh4Node (default) vs the previous commit (prev), and nearest-first-only ordering (s4off)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "tests=configs1 or window_bitexact or walk_handon or drain_continuation or configs0 or pipelines_bit or bvh_mode" \
  "vtests=s4off:configs1 or target_1m or walk_handon or drain_continuation or pipelines_bit or bvh_mode" \
  "abbench=3@--steps 20 --warmup 5@default,prev,s4off" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,prev,s4off" \
  "abbench=2@--accel bvh --steps 20 --warmup 5@default,prev,s4off"
