# VALU / SALU instruction counts (rocprofv3 SQ_INSTS_VALU + SQ_INSTS_SALU, kernel counters only)
# for bench.py's issue roofline: the bench's 16 pipelines (whole-job rate, tag _sq) and one
# pipeline (the per-kernel roofline pass, tag _sq_p1).  Writes gpurun_out/pmc_latest.json.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
cp profiles/pmc_latest.json gpurun_out/pmc_latest.json
for ACC in grid_fast bvh; do
  for P in 16 1; do
    B="bench.py --accel $ACC --alt-accel= --steps 8 --warmup 1 --no-cpu-baseline --no-profile --pipelines $P"
    timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/sq_${ACC}_p$P -o run --output-format csv -- python3 $B > gpurun_out/sq_${ACC}_p$P.log 2>&1 || { tail -20 gpurun_out/sq_${ACC}_p$P.log; exit 1; }
    T=_sq; [ $P = 1 ] && T=_sq_p1
    python3 scripts/pmc_summary.py sq ${ACC}_100000_1280x1024_b8 gpurun_out/sq_${ACC}_p$P 9 $T gpurun_out/pmc_latest.json > gpurun_out/sq_${ACC}_p$P.json || exit 1
  done
done
cp gpurun_out/pmc_latest.json profiles/pmc_latest.json
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_sq.json 2> gpurun_out/bench_sq.err; rc=$?
python3 -c "import json; d=json.load(open('gpurun_out/bench_sq.json')); print(d['value'], json.dumps(d['issue_roofline']))"; exit $rc
