# GPU suite + default A/B (VARIANTS) + optional stats-build variants (SVARIANTS)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python scripts/ab.py --rounds 3 --steps 4 --variants ${VARIANTS:-grid_fast:64} > gpurun_out/ab.json 2>/dev/null || exit 1
tr -d '\n ' < gpurun_out/ab.json; echo
if [ -n "$SVARIANTS" ]; then
  PT_LIB_PATH=$PWD/build_variants/lib_stats.so timeout -k 10 300 python scripts/ab.py --rounds 1 --steps 4 --variants $SVARIANTS > gpurun_out/abs.json 2>/dev/null || exit 1
  tr -d '\n ' < gpurun_out/abs.json; echo
fi
