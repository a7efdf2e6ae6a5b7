# walk_certify_fast with members cut to the near-side part the monotone walk can visit before s*
# (PT_CERT_NEAR=1, in-tree) vs the round-5 cut (build certold): parity subset on the in-tree library
# (including the certificate cross-check against the exact walk), certificate outcomes in stats builds,
# then interleaved library builds as separate processes.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
bash scripts/gpu_run.sh "tests=walk_certificates or walk_handon or member_box or voxel_boundary or configs1_bench or configs2_readme or configs4_10m_triangles_window or golden or drain_continuation or synthetic_scene" &&
PT_LIB_PATH=$PWD/build_variants/lib_statsnew.so timeout -k 10 300 python -u scripts/ab.py --rounds 1 --steps 4 --variants grid_fast:64:PT_DEBUG_ABLATE=2052 > gpurun_out/cert_statsnew.json 2> gpurun_out/cert_statsnew.err &&
PT_LIB_PATH=$PWD/build_variants/lib_statsold.so timeout -k 10 300 python -u scripts/ab.py --rounds 1 --steps 4 --variants grid_fast:64:PT_DEBUG_ABLATE=2052 > gpurun_out/cert_statsold.json 2> gpurun_out/cert_statsold.err &&
bash scripts/gpu_run.sh "ablib=3@grid_fast:64@default,certold" \
  "ablib=2@grid_fast:64 --ntri 10000000 --inmem --bounces 16@default,certold" \
  "ablib=2@grid_fast:64 --scene scenes/reference_scene.txt --width 2800 --height 2240 --bounces 5@default,certold"
