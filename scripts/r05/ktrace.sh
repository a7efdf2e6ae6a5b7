# kernel timelines of the bench's timed region (trace-kernel concurrency), configs[1] and configs[4]
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/gpu_run.sh "ktrace=--targets= --no-cpu-baseline --alt-accel= --no-profile --no-full-runs --steps 20 --warmup 5" \
  "ktrace=--targets= --no-cpu-baseline --alt-accel= --no-profile --no-full-runs --steps 16 --warmup 2 --ntri 10000000 --bounces 16 --inmem"
