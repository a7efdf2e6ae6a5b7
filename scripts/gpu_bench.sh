set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --steps 16 --warmup 2 > gpurun_out/bench_bvh.json 2> gpurun_out/bench_bvh.err || exit $?
cat gpurun_out/bench_bvh.json
timeout -k 10 400 python bench.py --accel grid --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_grid.json 2> gpurun_out/bench_grid.err || exit $?
cat gpurun_out/bench_grid.json
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1 -o bvh --output-format csv -- python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/prof_bvh.log 2>&1 || exit $?
find gpurun_out/prof_r1 -name "*stats*" | head
