# A/B: tail launches sized to their records (PT_TAIL_RPL), tail refill threshold, re-drain levels
# (parity subset first, then in-process interleaved timing at 10M / 16 bounces and 100k)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_render.py -x -q --timeout 120 --timeout-method thread -k "tail_sized or drain_continuation" > gpurun_out/tail_tests.log 2>&1 &&
timeout -k 10 600 python -u scripts/ab.py --inmem --ntri 10000000 --bounces 16 --rounds 3 --steps 16 --variants grid_fast:64 grid_fast:64:PT_TAIL_RPL=2 grid_fast:64:PT_TAIL_RPL=4 grid_fast:64:PT_TAIL_RPL=2,PT_TAIL_REFILL=16 grid_fast:64:PT_DRAIN_LEVELS=2 grid_fast:64:PT_DRAIN_LEVELS=2,PT_DRAIN_DUMP_TAIL=8,PT_TAIL_RPL=2 > gpurun_out/ab_tail10m.json 2> gpurun_out/ab_tail10m.err &&
timeout -k 10 600 python -u scripts/ab.py --rounds 3 --steps 20 --variants grid_fast:64 grid_fast:64:PT_TAIL_RPL=2 grid_fast:64:PT_TAIL_RPL=4 grid_fast:64:PT_TAIL_RPL=2,PT_TAIL_REFILL=16 grid_fast:64:PT_DRAIN_LEVELS=2 > gpurun_out/ab_tail100k.json 2> gpurun_out/ab_tail100k.err
