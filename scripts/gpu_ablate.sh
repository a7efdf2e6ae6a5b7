set -o pipefail
cd $GRAFT_REPO_ROOT
for A in 0 1 2; do
  PT_DEBUG_ABLATE=$A timeout -k 10 300 python scripts/ab.py --variants grid_fast:64 bvh:64 --rounds 2 --steps 8 > gpurun_out/ablate_$A.json 2>/dev/null || exit 1
  echo "ablate=$A $(python3 -c "import json;d=json.load(open('gpurun_out/ablate_$A.json'));print(' '.join(f'{k}={v[\"ms_per_spp_median\"]}' for k,v in d.items()))")"
done
