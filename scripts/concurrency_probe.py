#!/usr/bin/env python3
"""Probe: do two renderers on two HIP streams (separate pools, separate
images) trace more rays per second than one?  Interleaved rounds.

    python scripts/concurrency_probe.py --accel grid_fast --k 2
"""
import argparse
import os
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--accel", default="grid_fast")
    ap.add_argument("--k", type=int, default=2, help="concurrent renderers")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    import pathtracerap_amd as P
    from pathtracerap_amd import synthetic
    path = synthetic.diffuse_scene(tempfile.mkdtemp(), ntri=100_000)
    acc = {"bvh": P.ACCEL_BVH, "grid": P.ACCEL_GRID, "grid_fast": P.ACCEL_GRID_FAST}[a.accel]
    s = P.Scene(path)
    s.build(bvh=True)
    rs, streams = [], []
    for i in range(a.k):
        st = torch.cuda.Stream()
        r = P.Renderer(P.RenderConfig(width=1280, height=1024, max_bounces=8, accel=acc))
        r.set_stream(st.cuda_stream)
        r.allocateOnGPU(s)
        r.renderLoop(1000 + i, 1, sync=True)
        rs.append(r); streams.append(st)
    res = {"one": [], "all": []}
    for rnd in range(a.rounds):
        s0 = rs[0].segments(); torch.cuda.synchronize(); t = time.perf_counter()
        rs[0].renderLoop(rnd * 100, a.steps * a.k, sync=False); torch.cuda.synchronize()
        res["one"].append((rs[0].segments() - s0) / (time.perf_counter() - t) / 1e6)
        s0 = [r.segments() for r in rs]; torch.cuda.synchronize(); t = time.perf_counter()
        for i, r in enumerate(rs):
            r.renderLoop(rnd * 100 + 50 + i * a.steps, a.steps, sync=False)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        res["all"].append(sum(r.segments() - x for r, x in zip(rs, s0)) / dt / 1e6)
    print({k: round(statistics.median(v), 1) for k, v in res.items()}, "Mrays/s", a.accel, "k =", a.k)


if __name__ == "__main__":
    main()
