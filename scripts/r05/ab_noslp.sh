# the device code built without the SLP vectorizer (no packed-f32 shuffles): noslp; + k_trace_bvh at 5 waves per
# SIMD (nsb5, 90 VGPRs, no spills); + k_trace_gf at 5 waves (nsg5, 23 VGPRs spilled)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "vtests=noslp:configs1 or target_1m or window_bitexact or walk_handon or drain_continuation or configs0 or boundary or bvh_mode or pipelines_bit" \
  "abbench=3@--steps 20 --warmup 5@default,noslp,nsg5" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,noslp,nsg5" \
  "abbench=2@--accel bvh --steps 20 --warmup 5@default,noslp,nsb5"
