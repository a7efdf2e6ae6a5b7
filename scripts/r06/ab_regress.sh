# Where the round-6 code lost ~1 % against round 5: mesh-relative leaf links (PT_LEAF_REL=0:
# absolute) and the empty-mesh skip in the select steps (PT_EMPTY_SKIP=0), interleaved library
# builds; then all-phase iterations for few-lane waves (PT_ALLPHASE_LANES, in-process)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
bash scripts/gpu_run.sh "tests=tail_sized and 2" \
  "ablib=3@grid_fast:64@default,r05,abs,noempty,absnoempty" \
  "ablib=2@grid_fast:64 --ntri 10000000 --inmem --bounces 16@default,r05,absnoempty" \
  "ab=--rounds 3 --steps 20 --variants grid_fast:64 grid_fast:64:PT_ALLPHASE_LANES=16 grid_fast:64:PT_ALLPHASE_LANES=32 grid_fast:64:PT_ALLPHASE_LANES=64" \
  "ab=--inmem --ntri 10000000 --bounces 16 --rounds 2 --steps 16 --variants grid_fast:64 grid_fast:64:PT_ALLPHASE_LANES=16 grid_fast:64:PT_ALLPHASE_LANES=32 grid_fast:64:PT_ALLPHASE_LANES=64"
