# GPU parity tests against a variant library (PT_LIB_PATH), then an interleaved A/B of it
# against the in-tree library.  usage: gpu_testvar.sh NAME ROUNDS "VARIANT..."
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
N=$1; R=$2; V=$3
PT_LIB_PATH=$PWD/build_variants/lib_$N.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$N.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$N.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ablib.sh $R "$V" default $N
