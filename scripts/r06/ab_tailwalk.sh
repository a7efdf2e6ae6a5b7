# the tail's walk hand-ons skip the certificates the main launch already ran (state 7), and hand-on
# records copy only live stack entries and hit-set members (four loads in flight): parity subset, then
# interleaved library builds against the previous commit (base6)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
bash scripts/gpu_run.sh "tests=drain_continuation or walk_handon or tail_sized or allphase or pipelines or configs1_bench or iteration_4095 or configs4_10m_triangles_320" \
  "ablib=3@grid_fast:64@default,base6" \
  "ablib=2@grid_fast:64 --ntri 10000000 --inmem --bounces 16@default,base6" \
  "ablib=2@grid_fast:64 --ntri 1000000@default,base6" \
  "ablib=2@bvh:64@default,base6"
