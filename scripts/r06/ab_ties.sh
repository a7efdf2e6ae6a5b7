# walk_certify_fast accepting ties at t_min among members of one voxel box (the two triangles of a split
# quad): parity subset on the in-tree library (incl. the certificate cross-check against the exact walk and
# the full-size golden renders), certificate outcomes in the stats build, then interleaved library builds
# against the previous code (base7) as separate processes.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
bash scripts/gpu_run.sh "tests=walk_certificates or walk_handon or member_box or voxel_boundary or configs1_bench or configs2_readme or configs4_10m_triangles_window or golden or drain_continuation or synthetic_scene or iteration or configs0" &&
PT_LIB_PATH=$PWD/build_variants/lib_stats.so timeout -k 10 300 python -u scripts/ab.py --rounds 1 --steps 4 --variants grid_fast:64:PT_DEBUG_ABLATE=2052 > gpurun_out/stats_ties_100k.json 2> gpurun_out/stats_ties_100k.err &&
PT_LIB_PATH=$PWD/build_variants/lib_stats.so timeout -k 10 300 python -u scripts/ab.py --scene scenes/reference_scene.txt --width 2800 --height 2240 --bounces 5 --rounds 1 --steps 2 --variants grid_fast:64:PT_DEBUG_ABLATE=2052 > gpurun_out/stats_ties_c2.json 2> gpurun_out/stats_ties_c2.err &&
bash scripts/gpu_run.sh "ablib=3@grid_fast:64@default,base7" \
  "ablib=2@grid_fast:64 --ntri 10000000 --inmem --bounces 16@default,base7" \
  "ablib=2@grid_fast:64 --scene scenes/reference_scene.txt --width 2800 --height 2240 --bounces 5@default,base7"
