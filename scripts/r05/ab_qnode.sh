# 64-byte quantized 4-wide nodes in k_trace_gf (build_variants/lib_qn.so): parity subset, then A/B
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "vtests=qn:configs1 or target_1m or window_bitexact or walk_handon or drain_continuation or configs0 or configs2 or boundary" \
  "abbench=3@--steps 20 --warmup 5@default,qn" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,qn" \
  "abbench=2@--ntri 1000000 --steps 16 --warmup 2@default,qn" \
  "abbench=2@--scene scenes/reference_scene.txt --width 2800 --height 2240 --steps 16 --warmup 2@default,qn" \
  "abbench=2@--steps 20 --warmup 5 --pipelines 1@default,qn"
