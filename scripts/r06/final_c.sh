# Round-6 evidence at the final code: __graft_entry__.smoke(), the full GPU suite, the driver's bench line.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && cat gpurun_out/smoke.log &&
bash scripts/gpu_run.sh tests "bench=--steps 20 --warmup 5"
