# binned-SAH buckets per axis (host BLAS build): 8 / 32 vs 16
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "abbench=3@--steps 20 --warmup 5@default,bins32,bins8" \
  "abbench=2@--ntri 1000000 --steps 16 --warmup 2@default,bins32" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,bins32"
