# AMDGPU machine-scheduler strategies (sx1 max-ilp, sx2 max-memory-clause, sx3 iterative-ilp) and k_trace_bvh
# with three triangles per leaf step (bl3, 102 VGPRs), at the no-SLP build
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "abbench=3@--steps 20 --warmup 5@default,sx1,sx2,sx3" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,sx1,sx2,sx3" \
  "abbench=2@--accel bvh --steps 20 --warmup 5@default,sx1,sx2,bl3"
