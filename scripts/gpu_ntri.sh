# Scene-size sensitivity of the trace kernels: Mrays/s of grid_fast and bvh at
# several triangle counts (same camera / room; only the torus tessellation changes).
# usage: gpu_ntri.sh "10000 30000 100000 300000"
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for N in ${1:-10000 30000 100000 300000}; do
  timeout -k 10 300 python scripts/ab.py --variants grid_fast:64:PT_PIPES=16 bvh:64:PT_PIPES=16 --rounds 2 --steps 8 --ntri $N > gpurun_out/ntri_$N.json 2> gpurun_out/ntri_$N.err || { tail -5 gpurun_out/ntri_$N.err; exit 1; }
  echo "ntri $N"; cat gpurun_out/ntri_$N.json
done
