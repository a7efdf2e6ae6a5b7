# near / far planes loaded by the slope's sign in the 4-wide node steps (build_variants/lib_nf.so)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "vtests=nf:configs1 or target_1m or window_bitexact or walk_handon or drain_continuation or configs0 or boundary" \
  "abbench=3@--steps 20 --warmup 5@default,nf" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,nf" &&
bash scripts/gpu_run.sh "abbench=2@--accel bvh --steps 20 --warmup 5@default,bs2,bs3,bs6"
