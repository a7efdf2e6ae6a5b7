# A/B at the round-6 code: against the round-5 library (one BLAS on the device, mesh-relative
# leaves), LDS staging of the top 4-wide levels (PT_LDS_TOP 5 / 21 nodes, one or two meshes),
# depth-first node order (PT_BVH4_ORDER=1) and the skipped empty k_trace_deferred launch
# (PT_DEFER_LAUNCH=0); parity of the LDS variants on a GPU-test subset first
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
bash scripts/gpu_run.sh "vtests=ldstop21:trace_kernel_variants or walk_handon or configs1_bench" "vtests=ldstop5m1:trace_kernel_variants or walk_handon" \
  "ablib=3@grid_fast:64@default,r05,ldstop5m1,ldstop5,ldstop21" \
  "ablib=2@grid_fast:64 --ntri 10000000 --inmem --bounces 16@default,r05,ldstop5m1,ldstop21" \
  "ab=--rounds 3 --steps 20 --variants grid_fast:64 grid_fast:64:PT_BVH4_ORDER=1 grid_fast:64:PT_DEFER_LAUNCH=0" \
  "ab=--inmem --ntri 10000000 --bounces 16 --rounds 2 --steps 16 --variants grid_fast:64 grid_fast:64:PT_BVH4_ORDER=1 grid_fast:64:PT_DEFER_LAUNCH=0"
