#!/usr/bin/env python3
"""How long the host takes to enqueue a renderLoop call against how long the
GPU runs it: renderLoop(sync=False) returns once every launch is enqueued, so
its wall time is the host's enqueue time; synchronize() then gives the total.
A host that enqueues iteration i's ~64 launches while pipelines 0..i-1 already
run starts the last pipelines late (a ramp at the start of every call).

    python scripts/enqueue_probe.py [--ntri N] [--steps 16 20 32 64] [--graph]
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ntri", type=int, default=100_000)
    ap.add_argument("--bounces", type=int, default=8)
    ap.add_argument("--inmem", action="store_true")
    ap.add_argument("--steps", type=int, nargs="+", default=[16, 20, 32, 64])
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    import pathtracerap_amd as P
    from pathtracerap_amd import synthetic
    if a.inmem:
        s = synthetic.build_scene(P, ntri=a.ntri)
    else:
        s = P.Scene(synthetic.diffuse_scene(tempfile.mkdtemp(), ntri=a.ntri))
        s.build(bvh=True)
    r = P.Renderer(P.RenderConfig(width=1280, height=1024, max_bounces=a.bounces, accel=P.ACCEL_GRID_FAST))
    r.allocateOnGPU(s)
    r.renderLoop(0, 8)
    out = {"graph": os.environ.get("PT_GRAPH", "0"), "ntri": a.ntri}
    it = 100
    for k in a.steps:
        enq, tot = [], []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            r.synchronize()
            t0 = time.perf_counter()
            r.renderLoop(it, k, sync=False)
            t1 = time.perf_counter()
            r.synchronize()
            t2 = time.perf_counter()
            it += k
            enq.append((t1 - t0) * 1e3)
            tot.append((t2 - t0) * 1e3)
        out[str(k)] = {"enqueue_ms": round(min(enq), 3), "total_ms": round(min(tot), 3),
                       "ms_per_iter": round(min(tot) / k, 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
