# persistent grid_fast with in-kernel pool mode: GPU suite, variants, kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python scripts/ab.py --rounds 3 --steps 4 --variants grid_fast:64 grid_fast:64:PT_GF_SPLIT=0 > gpurun_out/ab.json 2>/dev/null || exit 1
echo "default $(tr -d '\n ' < gpurun_out/ab.json)"
for L in cap3 cap6 st8 st16; do
  PT_LIB_PATH=$PWD/build_variants/lib_$L.so timeout -k 10 200 python scripts/ab.py --variants grid_fast:64 --rounds 3 --steps 4 > gpurun_out/ab_$L.json 2>/dev/null || exit 1
  echo "$L $(tr -d '\n ' < gpurun_out/ab_$L.json)"
done
PT_LIB_PATH=$PWD/build_variants/lib_stats.so timeout -k 10 300 python scripts/ab.py --rounds 1 --steps 4 --variants grid_fast:64:PT_DEBUG_ABLATE=16 > gpurun_out/ab_gfst.json 2>/dev/null || exit 1
tr -d '\n ' < gpurun_out/ab_gfst.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kst -o run --output-format csv -- python3 scripts/ab.py --variants grid_fast:64 --rounds 1 --steps 4 > gpurun_out/kst.log 2>&1 || exit 1
python3 - <<'P'
import csv, glob
for f in glob.glob("gpurun_out/kst/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:60]:60s} {r['Calls']:>6} {float(r['AverageNs'])/1e3:10.1f} us {r['Percentage']}")
P
