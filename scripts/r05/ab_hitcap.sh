# k_trace_gf hit sets of 3 LDS members instead of 4 (hc3: 114 VGPRs, 1 KB less LDS per wave; more sets go to the global pool)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "vtests=hc3:configs1 or target_1m or window_bitexact or walk_handon or drain_continuation or configs0 or boundary" \
  "abbench=3@--steps 20 --warmup 5@default,hc3" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,hc3" \
  "abbench=2@--scene scenes/reference_scene.txt --width 2800 --height 2240 --bounces 5 --steps 8 --warmup 2@default,hc3"
