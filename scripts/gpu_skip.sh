# walk_skip + no-hit finality fix: old library on the new edge-miss test (expected to fail),
# full GPU suite on the new library, then A/B timing of old / noskip / new.
set -o pipefail
cd $GRAFT_REPO_ROOT
PT_LIB_PATH=$PWD/build_variants/lib_old.so timeout -k 10 120 python -u -m pytest tests/test_gpu_render.py -m gpu -q -k member_box_missed --timeout 60 --timeout-method thread > gpurun_out/old_edge.log 2>&1
echo "old-lib edge test rc=$? (1 = fails as expected)"; grep -E "passed|failed|Error" gpurun_out/old_edge.log | tail -4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for L in old noskip; do
  PT_LIB_PATH=$PWD/build_variants/lib_$L.so timeout -k 10 200 python scripts/ab.py --variants grid_fast:64 --rounds 3 --steps 4 > gpurun_out/ab_$L.json 2>/dev/null || exit 1
  echo "$L $(python3 -c "import json;d=json.load(open('gpurun_out/ab_$L.json'));print(d)")"
done
timeout -k 10 200 python scripts/ab.py --variants grid_fast:64 --rounds 3 --steps 4 > gpurun_out/ab_new.json 2>/dev/null || exit 1
echo "new $(cat gpurun_out/ab_new.json | tr -d '\n ')"
PT_LIB_PATH=$PWD/build_variants/lib_stats.so timeout -k 10 200 python scripts/ab.py --variants grid_fast:64:PT_DEBUG_ABLATE=4 --rounds 1 --steps 4 > gpurun_out/ab_stats.json 2>/dev/null || exit 1
cat gpurun_out/ab_stats.json
