# leaf triangle loads with 32-bit offsets (o32t); + s_setprio 1 / 3 around k_trace_gf's node and leaf steps (pr1, pr3)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "vtests=o32t:configs1 or target_1m or window_bitexact or walk_handon or drain_continuation or configs0 or bvh_mode" \
  "abbench=3@--steps 20 --warmup 5@default,o32t,pr1,pr3" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,o32t,pr1,pr3" \
  "abbench=2@--accel bvh --steps 20 --warmup 5@default,o32t"
