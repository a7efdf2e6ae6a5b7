# 64-byte quantized 4-wide nodes (qn), the fast certificate in the in-place walks (tfc), both (qntfc):
# parity subsets against the variant libraries, then interleaved A/B
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
K="configs1 or target_1m or window_bitexact or walk_handon or drain_continuation or configs0 or configs2 or pipelines_bit or boundary"
bash scripts/gpu_run.sh \
  "abbench=3@--steps 20 --warmup 5@default,qn,tfc,qntfc" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,qn,tfc,qntfc" \
  "abbench=2@--ntri 1000000 --steps 16 --warmup 2@default,qn,qntfc" \
  "abbench=2@--scene scenes/reference_scene.txt --width 2800 --height 2240 --steps 16 --warmup 2@default,qn,qntfc" \
  "abbench=2@--steps 20 --warmup 5 --pipelines 1@default,qn,tfc,qntfc"
