# Every GPU measurement of this repo, as named steps of one gpurun call.  Each
# step runs under its own time limit; the call stops at the first failure.
# Outputs go to gpurun_out/s<N>_<step>*.
#
#   usage: bash scripts/gpu_run.sh STEP [STEP ...]
#
#   tests[=EXPR]          pytest -m gpu (EXPR: a -k expression)
#   vtests=NAME:EXPR      the same against build_variants/lib_NAME.so (PT_LIB_PATH)
#   bench[=ARGS]          python bench.py ARGS (no ARGS: the driver's default line)
#   prof[=ARGS]           rocprofv3 --kernel-trace --stats of bench.py ARGS
#   ktrace[=ARGS]         rocprofv3 --kernel-trace of bench.py ARGS + scripts/timeline.py
#   pmc[=ARGS]            FETCH_SIZE and WRITE_SIZE, one --pmc pass each, of bench.py ARGS
#   counters=C1,C2@ARGS   one --pmc pass of the listed counters (within one pass's limits)
#   vcounters=LIB@C1,C2@ARGS  the same against build_variants/lib_LIB.so ("default" = in-tree)
#   ab=ARGS               python scripts/ab.py ARGS (interleaved in-process A/B)
#   ablib=R@SPEC@N1,N2    R interleaved rounds of ab.py SPEC over library builds
#                         (build_variants/lib_N.so from scripts/build_variant.sh; "default" = in-tree)
#   abbench=R@ARGS@N1,N2  R interleaved rounds of bench.py ARGS (main line only) over library builds
#   py=SCRIPT ARGS        python SCRIPT ARGS (a measurement script under scripts/)
#
# Example: bash scripts/gpu_run.sh tests "bench=--steps 32" "prof=--pipelines 1 --targets= --no-cpu-baseline"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-16}   # one hardware queue per pipeline stream (the library default too)
mkdir -p gpurun_out
n=0
for step in "$@"; do
  n=$((n + 1))
  name="${step%%=*}"; arg=""; [ "$name" != "$step" ] && arg="${step#*=}"
  tag="s${n}_${name}"
  echo "== step $n: $step"
  case "$name" in
    tests)
      if [ -n "$arg" ]; then
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$arg" > gpurun_out/$tag.log 2>&1
      else
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$tag.log 2>&1
      fi
      rc=$?; tail -15 gpurun_out/$tag.log ;;
    vtests)
      lib="${arg%%:*}"; k="${arg#*:}"
      PT_LIB_PATH=$PWD/build_variants/lib_$lib.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$k" > gpurun_out/$tag.log 2>&1
      rc=$?; tail -8 gpurun_out/$tag.log ;;
    bench)
      timeout -k 10 600 python -u bench.py $arg > gpurun_out/$tag.json 2> gpurun_out/$tag.err
      rc=$?; cat gpurun_out/$tag.json; tail -3 gpurun_out/$tag.err ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag -o run --output-format csv -- python3 bench.py $arg > gpurun_out/$tag.log 2>&1
      rc=$?; tail -2 gpurun_out/$tag.log ;;
    ktrace)
      timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/$tag -o run --output-format csv -- python3 bench.py $arg > gpurun_out/$tag.log 2>&1
      rc=$?; tail -2 gpurun_out/$tag.log
      [ $rc -eq 0 ] && { python3 scripts/timeline.py gpurun_out/$tag; rc=$?; } ;;
    pmc)
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${tag}_fetch -o run --output-format csv -- python3 bench.py $arg > gpurun_out/${tag}_fetch.log 2>&1
      rc=$?
      if [ $rc -eq 0 ]; then
        timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${tag}_write -o run --output-format csv -- python3 bench.py $arg > gpurun_out/${tag}_write.log 2>&1
        rc=$?
      fi
      tail -2 gpurun_out/${tag}_fetch.log ;;
    counters)
      c="${arg%%@*}"; a=""; [ "$c" != "$arg" ] && a="${arg#*@}"
      timeout -s KILL 300 rocprofv3 --pmc ${c//,/ } -d gpurun_out/$tag -o run --output-format csv -- python3 bench.py $a > gpurun_out/$tag.log 2>&1
      rc=$?; tail -2 gpurun_out/$tag.log
      [ $rc -eq 0 ] && { python3 scripts/pmc_table.py gpurun_out/$tag; rc=$?; } ;;
    vcounters)
      IFS=@ read -r lib c a <<< "$arg"
      if [ "$lib" = default ]; then L=$PWD/pathtracerap_amd/libpathtracer_amd.so; else L=$PWD/build_variants/lib_$lib.so; fi
      PT_LIB_PATH=$L timeout -s KILL 300 rocprofv3 --pmc ${c//,/ } -d gpurun_out/$tag -o run --output-format csv -- python3 bench.py $a > gpurun_out/$tag.log 2>&1
      rc=$?; tail -2 gpurun_out/$tag.log
      [ $rc -eq 0 ] && { python3 scripts/pmc_table.py gpurun_out/$tag > gpurun_out/$tag.txt; rc=$?; grep -A6 "k_trace_gf" gpurun_out/$tag.txt | head -20; } ;;
    ab)
      timeout -k 10 900 python -u scripts/ab.py $arg > gpurun_out/$tag.json 2> gpurun_out/$tag.err
      rc=$?; cat gpurun_out/$tag.json; tail -3 gpurun_out/$tag.err ;;
    ablib)
      IFS=@ read -r rounds spec names <<< "$arg"
      rc=0
      for r in $(seq 1 "$rounds"); do
        for lib in ${names//,/ }; do
          if [ "$lib" = default ]; then L=$PWD/pathtracerap_amd/libpathtracer_amd.so; else L=$PWD/build_variants/lib_$lib.so; fi
          PT_LIB_PATH=$L timeout -k 10 300 python scripts/ab.py --variants $spec --rounds 2 --steps 16 > gpurun_out/${tag}_$lib.json 2> gpurun_out/${tag}_$lib.err
          rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/${tag}_$lib.err; break 2; }
          python3 -c "import json; d=json.load(open('gpurun_out/${tag}_$lib.json')); print('round $r $lib', {k: v['Mrays_s'] for k, v in d.items()})" | tee -a gpurun_out/${tag}_rounds.txt
        done
      done ;;
    abbench)
      IFS=@ read -r rounds bargs names <<< "$arg"
      rc=0
      for r in $(seq 1 "$rounds"); do
        for lib in ${names//,/ }; do
          if [ "$lib" = default ]; then L=$PWD/pathtracerap_amd/libpathtracer_amd.so; else L=$PWD/build_variants/lib_$lib.so; fi
          PT_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --alt-accel= --targets= $bargs > gpurun_out/${tag}_$lib.json 2> gpurun_out/${tag}_$lib.err
          rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/${tag}_$lib.err; break 2; }
          python3 -c "import json; d=json.load(open('gpurun_out/${tag}_$lib.json')); print('round $r $lib', d['value'], d['ms_per_step'])" | tee -a gpurun_out/${tag}_rounds.txt
        done
      done ;;
    py)
      timeout -k 10 900 python -u $arg > gpurun_out/$tag.log 2>&1
      rc=$?; tail -25 gpurun_out/$tag.log ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
  [ $rc -eq 0 ] || { echo "step $step failed rc=$rc"; exit $rc; }
done
