# PT_HIT_LATE=1 (build variant): a finished ray's hit record waits in the lane's first hit-set slot and is
# stored behind the next refill's claim atomic, so the claim does not wait on the store (vmcnt counts
# stores on gfx950).  Parity subset against the variant first, then interleaved library builds.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
bash scripts/gpu_run.sh "vtests=hitlate:drain_continuation or walk_handon or tail_sized or pipelines_bit_identical or bench_configuration or main_launch_sized" \
  "ablib=3@grid_fast:64@default,hitlate" \
  "ablib=2@grid_fast:64 --ntri 10000000 --inmem --bounces 16@default,hitlate"
