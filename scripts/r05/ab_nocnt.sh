# 4-wide node steps without the count float4 (empty slots are inverted infinite boxes): build_variants/lib_nc0.so
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "vtests=nc0:configs1 or target_1m or window_bitexact or walk_handon or drain_continuation or configs0 or boundary or bvh_mode or pipelines_bit" \
  "abbench=3@--steps 20 --warmup 5@default,nc0" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,nc0" \
  "abbench=2@--accel bvh --steps 20 --warmup 5@default,nc0"
