# full walk certificate deferred until 4 / 8 lanes need it (build_variants/lib_df4.so, lib_df8.so)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "vtests=df4:configs1 or target_1m or window_bitexact or walk_handon or drain_continuation or configs0 or boundary or certif" \
  "abbench=3@--steps 20 --warmup 5@default,df4,df8" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,df4,df8" \
  "abbench=2@--scene scenes/reference_scene.txt --width 2800 --height 2240 --bounces 5 --steps 8 --warmup 2@default,df4,df8"
