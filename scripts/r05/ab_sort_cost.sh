# A/B: cost-class claim order (PT_SORT 9 / 10) against the default key 7, interleaved in one process
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && mkdir -p gpurun_out &&
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ray_sort_bit_identical" > gpurun_out/t_sort.log 2>&1 && tail -2 gpurun_out/t_sort.log &&
timeout -k 10 600 python -u scripts/ab.py --inmem --ntri 10000000 --bounces 16 --rounds 3 --steps 8 --variants grid_fast:64 grid_fast:64:PT_SORT=9 grid_fast:64:PT_SORT=10 > gpurun_out/ab_sort10m.json 2> gpurun_out/ab_sort10m.err &&
timeout -k 10 600 python -u scripts/ab.py --rounds 3 --steps 16 --variants grid_fast:64 grid_fast:64:PT_SORT=9 grid_fast:64:PT_SORT=10 > gpurun_out/ab_sort100k.json 2> gpurun_out/ab_sort100k.err &&
timeout -k 10 600 python -u scripts/ab.py --ntri 1000000 --rounds 3 --steps 16 --variants grid_fast:64 grid_fast:64:PT_SORT=9 grid_fast:64:PT_SORT=10 > gpurun_out/ab_sort1m.json 2> gpurun_out/ab_sort1m.err
