# PT_CERT_MODE=2 (build variant): k_trace_gf's main launch runs only the fast walk certificate; a hit set
# it declines is handed on to the tail, which walks it exactly (since round 6 without re-running the
# certificates).  Round 5 measured -5 % at the README scene -- before the tail skipped the certificates
# and while that scene's walk hand-ons overflowed their room into k_trace_deferred.  Parity subset
# against the variant, then interleaved library builds as separate processes.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
bash scripts/gpu_run.sh "vtests=cert2:drain_continuation or walk_handon or tail_sized or tail_grid or configs1_bench or bench_configuration or member_box or voxel_boundary or configs2" \
  "ablib=3@grid_fast:64@default,cert2" \
  "ablib=2@grid_fast:64 --ntri 10000000 --inmem --bounces 16@default,cert2" \
  "ablib=2@grid_fast:64 --scene scenes/reference_scene.txt --width 2800 --height 2240 --bounces 5@default,cert2"
