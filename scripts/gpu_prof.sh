# rocprofv3 kernel trace + stats of the default bench command, then grid-mode bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1 -o bvh --output-format csv -- python3 bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bvh.log 2>&1
rc=$?; tail -3 gpurun_out/prof_bvh.log; [ $rc -eq 0 ] || exit $rc
find gpurun_out/prof_r1 -type f | head -20
timeout -k 10 600 python bench.py --accel grid --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_grid.json 2> gpurun_out/bench_grid.err
rc=$?; cat gpurun_out/bench_grid.json; exit $rc
