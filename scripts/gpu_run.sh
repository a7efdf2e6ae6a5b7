# One GPU call, steps chosen by name (each under its own time limit, stopping at
# the first failure).  Outputs under gpurun_out/.
#   usage: bash scripts/gpu_run.sh STEP [STEP ...]
#   tests[=EXPR]     pytest -m gpu (optional -k EXPR)
#   bench[=ARGS]     python bench.py ARGS (default: the driver's default line)
#   prof[=ARGS]      rocprofv3 --kernel-trace --stats of bench.py ARGS
#   pmc[=ARGS]       separate FETCH_SIZE / WRITE_SIZE passes of bench.py ARGS
#   sq[=ARGS]        SQ_INSTS_VALU / SQ_INSTS_SALU pass of bench.py ARGS
#   py=SCRIPT        python SCRIPT (a measurement script under scripts/)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
n=0
for step in "$@"; do
  n=$((n + 1))
  name="${step%%=*}"; arg=""; [ "$name" != "$step" ] && arg="${step#*=}"
  tag="s${n}_${name}"
  case "$name" in
    tests)
      k=""; [ -n "$arg" ] && k="-k $arg"
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $k > gpurun_out/$tag.log 2>&1
      rc=$?; tail -15 gpurun_out/$tag.log ;;
    bench)
      timeout -k 10 600 python -u bench.py $arg > gpurun_out/$tag.json 2> gpurun_out/$tag.err
      rc=$?; cat gpurun_out/$tag.json; tail -3 gpurun_out/$tag.err ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag -o run --output-format csv -- python3 bench.py $arg > gpurun_out/$tag.log 2>&1
      rc=$?; tail -3 gpurun_out/$tag.log ;;
    pmc)
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${tag}_fetch -o run --output-format csv -- python3 bench.py $arg > gpurun_out/${tag}_fetch.log 2>&1
      rc=$?
      [ $rc -eq 0 ] && { timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${tag}_write -o run --output-format csv -- python3 bench.py $arg > gpurun_out/${tag}_write.log 2>&1; rc=$?; }
      tail -3 gpurun_out/${tag}_fetch.log ;;
    sq)
      timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/$tag -o run --output-format csv -- python3 bench.py $arg > gpurun_out/$tag.log 2>&1
      rc=$?; tail -3 gpurun_out/$tag.log ;;
    py)
      timeout -k 10 900 python -u $arg > gpurun_out/$tag.log 2>&1
      rc=$?; tail -20 gpurun_out/$tag.log ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
  [ $rc -eq 0 ] || { echo "step $step failed rc=$rc"; exit $rc; }
done
