# Round-6 evidence, call A: __graft_entry__.smoke(), the full GPU suite, the driver's bench line, then the
# configs[1] profile set (scripts/round_profiles.sh 1).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && cat gpurun_out/smoke.log &&
bash scripts/gpu_run.sh tests "bench=--steps 20 --warmup 5" &&
cp gpurun_out/s1_tests.log gpurun_out/final_tests.log && cp gpurun_out/s2_bench.json gpurun_out/final_bench.json &&
bash scripts/round_profiles.sh 1
