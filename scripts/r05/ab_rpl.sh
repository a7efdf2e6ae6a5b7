# A/B: main trace launches sized to the bounce's rays (PT_TRACE_RPL rays per lane), interleaved in one process
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
timeout -k 10 600 python -u scripts/ab.py --inmem --ntri 10000000 --bounces 16 --rounds 3 --steps 8 --variants grid_fast:64 grid_fast:64:PT_TRACE_RPL=2 grid_fast:64:PT_TRACE_RPL=4 grid_fast:64:PT_TRACE_RPL=8 grid_fast:64:PT_TRACE_RPL=16 > gpurun_out/ab_rpl10m.json 2> gpurun_out/ab_rpl10m.err &&
timeout -k 10 600 python -u scripts/ab.py --rounds 3 --steps 16 --variants grid_fast:64 grid_fast:64:PT_TRACE_RPL=2 grid_fast:64:PT_TRACE_RPL=4 grid_fast:64:PT_TRACE_RPL=8 grid_fast:64:PT_TRACE_RPL=16 > gpurun_out/ab_rpl100k.json 2> gpurun_out/ab_rpl100k.err &&
timeout -k 10 600 python -u scripts/ab.py --ntri 1000000 --rounds 3 --steps 16 --variants grid_fast:64 grid_fast:64:PT_TRACE_RPL=4 grid_fast:64:PT_TRACE_RPL=8 > gpurun_out/ab_rpl1m.json 2> gpurun_out/ab_rpl1m.err
