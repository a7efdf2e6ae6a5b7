# GPU parity tests on the in-tree library, then an interleaved A/B of library builds.
# usage: gpu_testab.sh ROUNDS "VARIANT..." NAME...   (see gpu_ablib.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ablib.sh "$@"
