# fewer main-launch waves for sparse bounces (PT_TRACE_MIN_WAVES_PER_CU 1, PT_TRACE_RPL 8) and 20 pipelines, combined
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
V="grid_fast:64 grid_fast:64:PT_TRACE_MIN_WAVES_PER_CU=1 grid_fast:64:PT_TRACE_RPL=8 grid_fast:64:PT_TRACE_MIN_WAVES_PER_CU=1,PT_TRACE_RPL=8 grid_fast:64:PT_PIPES=20 grid_fast:64:PT_PIPES=20,PT_TRACE_MIN_WAVES_PER_CU=1" &&
timeout -k 10 600 python -u scripts/ab.py --rounds 5 --steps 20 --variants $V > gpurun_out/ab_rth100k.json 2> gpurun_out/ab_rth100k.err &&
timeout -k 10 600 python -u scripts/ab.py --ntri 1000000 --rounds 3 --steps 16 --variants $V > gpurun_out/ab_rth1m.json 2> gpurun_out/ab_rth1m.err &&
timeout -k 10 600 python -u scripts/ab.py --inmem --ntri 10000000 --bounces 16 --rounds 3 --steps 16 --variants $V > gpurun_out/ab_rth10m.json 2> gpurun_out/ab_rth10m.err
