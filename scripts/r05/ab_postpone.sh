# postponed leaves in the 4-wide node steps (build_variants/lib_pp.so): parity subset, then A/B
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "vtests=pp:configs1 or target_1m or window_bitexact or walk_handon or drain_continuation or pipelines_bit_identical or configs0 or configs2" \
  "abbench=3@--steps 20 --warmup 5@default,pp" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,pp" \
  "abbench=2@--ntri 1000000 --steps 16 --warmup 2@default,pp" \
  "abbench=2@--scene scenes/reference_scene.txt --width 2800 --height 2240 --steps 16 --warmup 2@default,pp" \
  "abbench=2@--steps 20 --warmup 5 --pipelines 1@default,pp"
