# A/B: trace launch sizing at the round-6 code -- waves per CU of a persistent launch
# (PT_TRACE_WAVES_PER_CU), rays per lane of sparse bounces (PT_TRACE_RPL), pipelines (PT_PIPES).
# Runtime settings only (same library, in-process interleaved); results are unchanged by construction
# (which wave traces which ray), as tests/test_gpu_render.py's tail/pipeline cases pin.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
timeout -k 10 700 python -u scripts/ab.py --inmem --ntri 10000000 --bounces 16 --rounds 2 --steps 16 --variants grid_fast:64 grid_fast:64:PT_TRACE_WAVES_PER_CU=4 grid_fast:64:PT_TRACE_WAVES_PER_CU=6 grid_fast:64:PT_TRACE_WAVES_PER_CU=12 grid_fast:64:PT_TRACE_RPL=8 grid_fast:64:PT_TRACE_RPL=8,PT_TRACE_WAVES_PER_CU=6 grid_fast:64:PT_PIPES=12 grid_fast:64:PT_PIPES=12,PT_TRACE_WAVES_PER_CU=12 > gpurun_out/ab_sizing10m.json 2> gpurun_out/ab_sizing10m.err &&
timeout -k 10 500 python -u scripts/ab.py --rounds 3 --steps 20 --variants grid_fast:64 grid_fast:64:PT_TRACE_WAVES_PER_CU=4 grid_fast:64:PT_TRACE_WAVES_PER_CU=6 grid_fast:64:PT_TRACE_WAVES_PER_CU=12 grid_fast:64:PT_TRACE_RPL=8 grid_fast:64:PT_PIPES=12,PT_TRACE_WAVES_PER_CU=12 > gpurun_out/ab_sizing100k.json 2> gpurun_out/ab_sizing100k.err
