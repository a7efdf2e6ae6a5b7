# Full round check on one MI355X: GPU parity tests, rocprofv3 kernel stats
# (default bench = 8 pipelines, and --pipelines 1 whose per-launch durations are
# the roofline's), PMC passes (FETCH_SIZE / WRITE_SIZE separately, one pipeline)
# for grid_fast and bvh, then the default bench line.
# usage: gpu_round.sh   (outputs under gpurun_out/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
cp profiles/pmc_latest.json gpurun_out/pmc_latest.json
for ACC in grid_fast bvh; do
  B="bench.py --accel $ACC --alt-accel= --steps 8 --warmup 1 --no-cpu-baseline --no-profile"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$ACC -o run --output-format csv -- python3 $B > gpurun_out/prof_$ACC.log 2>&1 || { tail -20 gpurun_out/prof_$ACC.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1_$ACC -o run --output-format csv -- python3 bench.py --accel $ACC --alt-accel= --steps 32 --warmup 2 --no-cpu-baseline --no-profile --pipelines 1 > gpurun_out/prof1_$ACC.log 2>&1 || { tail -20 gpurun_out/prof1_$ACC.log; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$ACC -o run --output-format csv -- python3 $B --pipelines 1 > gpurun_out/pmc_fetch_$ACC.log 2>&1 || { tail -20 gpurun_out/pmc_fetch_$ACC.log; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$ACC -o run --output-format csv -- python3 $B --pipelines 1 > gpurun_out/pmc_write_$ACC.log 2>&1 || { tail -20 gpurun_out/pmc_write_$ACC.log; exit 1; }
  python3 scripts/pmc_summary.py ${ACC}_100000_1280x1024_b8 gpurun_out/pmc_fetch_$ACC gpurun_out/pmc_write_$ACC gpurun_out/pmc_latest.json > /dev/null || exit 1
done
cp gpurun_out/pmc_latest.json profiles/pmc_latest.json
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; exit $rc
