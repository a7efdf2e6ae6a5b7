# 4-wide BLAS in k_trace_gf (build_variants/lib_bvh4.so, -DPT_GF_BVH4=1): parity subset, then interleaved A/B
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "vtests=bvh4:configs1 or target_1m or window_bitexact or walk_handon or drain_continuation or pipelines_bit_identical or configs0" \
  "abbench=3@--steps 20 --warmup 5@default,bvh4" "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,bvh4" \
  "abbench=2@--ntri 1000000 --steps 16 --warmup 2@default,bvh4"
