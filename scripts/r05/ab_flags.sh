# codegen flags on top of -fno-slp-vectorize: -fno-vectorize (nv), -fno-unroll-loops (nu), both (nvnu)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "vtests=nvnu:configs1 or target_1m or window_bitexact or walk_handon or drain_continuation or configs0 or bvh_mode" \
  "abbench=3@--steps 20 --warmup 5@default,nv,nu,nvnu" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,nv,nu,nvnu" \
  "abbench=2@--accel bvh --steps 20 --warmup 5@default,nv,nu,nvnu"
