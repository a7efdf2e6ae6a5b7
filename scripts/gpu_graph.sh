# hipGraph replay (PT_GRAPH=1): parity tests, then an interleaved A/B against direct launches.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_render.py -k "graph or pipelines or bench_configuration" -x -v --timeout 120 --timeout-method thread > gpurun_out/graph_test.log 2>&1
rc=$?; tail -12 gpurun_out/graph_test.log; [ $rc -eq 0 ] || exit $rc
GPU_MAX_HW_QUEUES=16 timeout -k 10 600 python scripts/ab.py --variants grid_fast:64:PT_PIPES=16 grid_fast:64:PT_PIPES=16,PT_GRAPH=1 bvh:64:PT_PIPES=16 bvh:64:PT_PIPES=16,PT_GRAPH=1 grid_fast:64:PT_PIPES=8,PT_GRAPH=1 --rounds 3 --steps 16 > gpurun_out/ab_graph.json 2> gpurun_out/ab_graph.err
rc=$?; cat gpurun_out/ab_graph.json; tail -3 gpurun_out/ab_graph.err; exit $rc
