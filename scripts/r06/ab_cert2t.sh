# With ties handled by the fast certificate (99.4 % accepted at configs[1]), the full certificate rescues
# 0.09 % of walks in the main launch: the fast certificate alone there (PT_CERT_MODE=2, build cert2t; the
# rest handed on to the tail's exact walk) against the in-tree default.  Parity subset against the variant
# first, then interleaved library builds as separate processes.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
bash scripts/gpu_run.sh "vtests=cert2t:walk_handon or member_box or voxel_boundary or configs1_bench or configs2_readme or configs4_10m_triangles_window or golden or drain_continuation or synthetic_scene or iteration" \
  "ablib=3@grid_fast:64@default,cert2t" \
  "ablib=2@grid_fast:64 --ntri 10000000 --inmem --bounces 16@default,cert2t" \
  "ablib=2@grid_fast:64 --scene scenes/reference_scene.txt --width 2800 --height 2240 --bounces 5@default,cert2t"
