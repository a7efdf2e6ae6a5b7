# ab.py with a global env (e.g. PT_DEBUG_ABLATE) for all variants.  usage: gpu_abenv.sh "ENV=.." variants...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
E=$1; shift
env $E timeout -k 10 400 python scripts/ab.py --variants "$@" --rounds 1 --steps 2 > gpurun_out/abenv.json 2>gpurun_out/abenv.err || { tail -5 gpurun_out/abenv.err; exit 1; }
cat gpurun_out/abenv.json
