# walk phase at the 4-wide default: fast certificate only in the main launch (PT_CERT_MODE 2), walk weights
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "abbench=3@--steps 20 --warmup 5@default,cm2,ww12,ww16,ww24" \
  "abbench=2@--ntri 10000000 --bounces 16 --inmem --steps 16 --warmup 2@default,cm2,ww16" \
  "abbench=2@--scene scenes/reference_scene.txt --width 2800 --height 2240 --steps 16 --warmup 2@default,cm2,ww16"
