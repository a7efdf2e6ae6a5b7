# Round profile: kernel trace + stats, PMC passes (FETCH_SIZE / WRITE_SIZE separately), then the bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ACC=${1:-grid_fast}
B="bench.py --accel $ACC --alt-accel= --steps 8 --warmup 1 --no-cpu-baseline --no-profile"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$ACC -o run --output-format csv -- python3 $B > gpurun_out/prof_$ACC.log 2>&1 || { tail -20 gpurun_out/prof_$ACC.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$ACC -o run --output-format csv -- python3 $B > gpurun_out/pmc_fetch.log 2>&1 || { tail -20 gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$ACC -o run --output-format csv -- python3 $B > gpurun_out/pmc_write.log 2>&1 || { tail -20 gpurun_out/pmc_write.log; exit 1; }
cp profiles/pmc_latest.json gpurun_out/pmc_latest.json
python3 scripts/pmc_summary.py ${ACC}_100000_1280x1024_b8 gpurun_out/pmc_fetch_$ACC gpurun_out/pmc_write_$ACC gpurun_out/pmc_latest.json || exit 1
cp gpurun_out/pmc_latest.json profiles/pmc_latest.json
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; exit $rc
