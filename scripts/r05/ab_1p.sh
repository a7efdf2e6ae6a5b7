# one pipeline (the roofline pass's setting): refill threshold (in-process interleaved)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
timeout -k 10 600 python -u scripts/ab.py --rounds 3 --steps 12 --variants grid_fast:64:PT_PIPES=1 grid_fast:64:PT_PIPES=1,PT_TRACE_REFILL=40 grid_fast:64:PT_PIPES=1,PT_TRACE_REFILL=48 grid_fast:64:PT_PIPES=1,PT_TRACE_REFILL=56 grid_fast:64:PT_PIPES=1,PT_TRACE_REFILL=64 > gpurun_out/ab_1p2.json 2> gpurun_out/ab_1p2.err &&
timeout -k 10 600 python -u scripts/ab.py --inmem --ntri 10000000 --bounces 16 --rounds 2 --steps 8 --variants grid_fast:64:PT_PIPES=1 grid_fast:64:PT_PIPES=1,PT_TRACE_REFILL=48 grid_fast:64:PT_PIPES=1,PT_TRACE_REFILL=56 > gpurun_out/ab_1p3.json 2> gpurun_out/ab_1p3.err
