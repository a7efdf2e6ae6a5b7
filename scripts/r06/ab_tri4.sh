# PT_TRI_REC=4 (build variant): 64-byte leaf triangle records and two-triangle leaves aligned to one
# 128-byte line (48-byte records: 5 of 8 such leaves straddle two lines).  Parity subset against the
# variant (both BLAS traces, the one-lane paths, the benched sizes), then interleaved library builds as
# separate processes.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
bash scripts/gpu_run.sh "vtests=tri4:synthetic_scene or intersect_random or bvh_matches or drain_continuation or tail_sized or pipelines_bit_identical or configs1_bench or target_1m_triangles or bvh_mode_window or configs4_10m_triangles_window or member_box or voxel_boundary" \
  "ablib=3@grid_fast:64@default,tri4" \
  "ablib=2@grid_fast:64 --ntri 10000000 --inmem --bounces 16@default,tri4" \
  "ablib=2@grid_fast:64 --ntri 1000000@default,tri4" \
  "ablib=2@bvh:64@default,tri4" &&
# ray sort keys re-swept at the 4-wide code (PT_SORT: 7 default, 1 direction-major, 2 origin-major, 6 origin
# 8^3 + octant, 8 direction 16x16 interleaved); in-process, 3 rounds (median)
timeout -k 10 300 python -u scripts/ab.py --rounds 3 --steps 20 --variants grid_fast:64 grid_fast:64:PT_SORT=1 grid_fast:64:PT_SORT=2 grid_fast:64:PT_SORT=6 grid_fast:64:PT_SORT=8 > gpurun_out/ab_sort100k.json 2> gpurun_out/ab_sort100k.err &&
timeout -k 10 300 python -u scripts/ab.py --inmem --ntri 10000000 --bounces 16 --rounds 3 --steps 16 --variants grid_fast:64 grid_fast:64:PT_SORT=2 grid_fast:64:PT_SORT=6 grid_fast:64:PT_SORT=8 > gpurun_out/ab_sort10m.json 2> gpurun_out/ab_sort10m.err
