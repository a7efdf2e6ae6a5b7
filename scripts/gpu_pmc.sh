# PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs) + the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-profile"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 $B > gpurun_out/pmc_fetch.log 2>&1 || { tail -20 gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 $B > gpurun_out/pmc_write.log 2>&1 || { tail -20 gpurun_out/pmc_write.log; exit 1; }
python3 scripts/pmc_summary.py bvh_100000_1280x1024_b8 gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_latest.json || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench_bvh.json 2> gpurun_out/bench_bvh.err
rc=$?; cat gpurun_out/bench_bvh.json; tail -3 gpurun_out/bench_bvh.err; exit $rc
