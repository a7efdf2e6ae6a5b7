# drain threshold at the 4-wide code, 10M and 100k (in-process interleaved)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
timeout -k 10 600 python -u scripts/ab.py --inmem --ntri 10000000 --bounces 16 --rounds 2 --steps 16 --variants grid_fast:64 grid_fast:64:PT_DRAIN_DUMP=0 grid_fast:64:PT_DRAIN_DUMP=8 grid_fast:64:PT_DRAIN_DUMP=32 grid_fast:64:PT_DRAIN_DUMP=48 > gpurun_out/ab_dr10m.json 2> gpurun_out/ab_dr10m.err &&
timeout -k 10 600 python -u scripts/ab.py --rounds 3 --steps 20 --variants grid_fast:64 grid_fast:64:PT_DRAIN_DUMP=0 grid_fast:64:PT_DRAIN_DUMP=32 > gpurun_out/ab_dr100k.json 2> gpurun_out/ab_dr100k.err
