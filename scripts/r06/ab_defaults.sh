# New defaults (rays per lane 8 when the BLAS exceeds the aggregate L2; walk hand-on room >= one per 16
# pixels) against the old ones, after the parity subset: the A/B variants with PT_TRACE_RPL=4 /
# PT_WALK_WCAP=131072 are the round-6 code before the change (trace_blocks * 64 = 131072 at 16 pipelines).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_render.py -x -v --timeout 200 --timeout-method thread -k "main_launch_sized or walk_handon or drain_continuation or tail_sized or pipelines_bit_identical or bench_configuration" > gpurun_out/defaults_tests.log 2>&1 &&
timeout -k 10 500 python -u scripts/ab.py --rounds 3 --steps 20 --variants grid_fast:64 grid_fast:64:PT_TRACE_RPL=2 grid_fast:64:PT_TRACE_RPL=3 grid_fast:64:PT_TRACE_RPL=6 > gpurun_out/ab_def100k.json 2> gpurun_out/ab_def100k.err &&
timeout -k 10 500 python -u scripts/ab.py --ntri 1000000 --rounds 3 --steps 16 --variants grid_fast:64 grid_fast:64:PT_TRACE_RPL=4 grid_fast:64:PT_TRACE_RPL=6 grid_fast:64:PT_TRACE_RPL=12 > gpurun_out/ab_def1m.json 2> gpurun_out/ab_def1m.err &&
timeout -k 10 500 python -u scripts/ab.py --inmem --ntri 10000000 --bounces 16 --rounds 3 --steps 16 --variants grid_fast:64 grid_fast:64:PT_TRACE_RPL=4 > gpurun_out/ab_def10m.json 2> gpurun_out/ab_def10m.err &&
timeout -k 10 500 python -u scripts/ab.py --scene scenes/reference_scene.txt --width 2800 --height 2240 --bounces 5 --rounds 3 --steps 12 --variants grid_fast:64 grid_fast:64:PT_WALK_WCAP=131072 > gpurun_out/ab_defc2.json 2> gpurun_out/ab_defc2.err
