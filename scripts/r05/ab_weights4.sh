# phase weights at the 4-wide code: leaf 2 / 5 vs 3, select 2 / 6 vs 4
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "abbench=3@--steps 20 --warmup 5@default,lw2,lw5,sw2,sw6" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,lw2,lw5"
