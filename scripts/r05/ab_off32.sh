# node loads from the SGPR base + 32-bit offsets (o32), + 32-bit spill indexing (o32s)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "vtests=o32s:configs1 or target_1m or window_bitexact or walk_handon or drain_continuation or configs0 or boundary or bvh_mode or pipelines_bit" \
  "abbench=3@--steps 20 --warmup 5@default,o32,o32s" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,o32,o32s" \
  "abbench=2@--accel bvh --steps 20 --warmup 5@default,o32,o32s"
