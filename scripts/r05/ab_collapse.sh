# 4-wide collapse: greedy largest-area opening (default) vs opening both children once (HEAD c2 build);
# then BLAS leaf size at the 4-wide default (one process per setting)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "abbench=3@--steps 20 --warmup 5@default,c2" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,c2" \
  "abbench=2@--ntri 1000000 --steps 16 --warmup 2@default,c2" \
  "abbench=2@--accel bvh --steps 20 --warmup 5@default,c2" &&
bash scripts/envsweep.sh 2 "--steps 20 --warmup 5" "" "PT_BVH_LEAF=1" "PT_BVH_LEAF=3" "PT_BVH_LEAF=4"
