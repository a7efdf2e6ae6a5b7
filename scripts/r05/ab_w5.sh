# k_trace_gf at 5 waves per SIMD (<= 96 VGPRs, LDS <= 8 KB per wave: hit-set cap 3 or LDS stack 8) vs 4
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "abbench=3@--steps 20 --warmup 5@default,w5a,w5b,hc3" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,w5a,w5b"
