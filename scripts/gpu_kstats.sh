# rocprofv3 kernel stats for one ab.py variant.  usage: gpu_kstats.sh VARIANT
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kst -o run --output-format csv -- python3 scripts/ab.py --variants "$1" --rounds 1 --steps 4 > gpurun_out/kst.log 2>&1 || { tail -5 gpurun_out/kst.log; exit 1; }
python3 - <<'P'
import csv, glob
for f in glob.glob("gpurun_out/kst/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:60]:60s} {r['Calls']:>6} {float(r['AverageNs'])/1e3:10.1f} us {r['Percentage']}")
P
