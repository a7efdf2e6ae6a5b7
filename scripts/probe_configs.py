"""Timing probe for the BASELINE-size parity tests (GPU box): scene builds,
grid_fast / grid renders and oracle renders at configs[1], the 1M target,
configs[2] and configs[4] sizes.  Prints one line per measurement."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
import pathtracerap_amd as P  # noqa: E402
from pathtracerap_amd import synthetic  # noqa: E402
from helpers import flat_from_export, oracle_cfg  # noqa: E402

O.build()


def t_gpu(s, cfg, label):
    t = time.time()
    r = P.Renderer(cfg)
    r.allocateOnGPU(s)
    r.renderLoop()
    img = r.image()
    pb = r.segments_per_bounce(20)
    print(f"{label}: gpu {time.time() - t:.2f}s segs {r.segments()} faults {r.trace_faults()} "
          f"deferred {r.deferred_rays()} per_bounce {pb}", flush=True)
    r.free()
    return img, pb


def t_oracle(s, cfg, label):
    t = time.time()
    img, seg = O.render(flat_from_export(s.export(), cfg.grid), oracle_cfg(cfg, threads=16))
    print(f"{label}: oracle {time.time() - t:.2f}s segs {seg}", flush=True)
    return img


which = sys.argv[1:] or ["10m"]
if "10m" in which:
    t = time.time()
    s = synthetic.build_scene(P, ntri=10_000_000)
    print("10m build", time.time() - t, s.counts(), flush=True)
    for w, h in ((320, 256), (1280, 1024)):
        cfg = P.RenderConfig(width=w, height=h, iterations=1, max_bounces=16)
        a, pa = t_gpu(s, cfg, f"10m grid_fast {w}x{h}")
        if w == 320:
            cfg.accel = P.ACCEL_GRID
            b, pb = t_gpu(s, cfg, f"10m grid {w}x{h}")
            print("equal", np.array_equal(a.view(np.uint32), b.view(np.uint32)), pa == pb, flush=True)
    cfg = P.RenderConfig(width=64, height=64, iterations=1, max_bounces=16, plane_x0=5.0, plane_y0=2.5,
                         plane_w=1.0, plane_h=1.0)
    a, _ = t_gpu(s, cfg, "10m crop")
    o = t_oracle(s, cfg, "10m crop")
    print("crop equal", np.array_equal(a.view(np.uint32), o.view(np.uint32)), flush=True)
if "1m" in which:
    import tempfile
    d = tempfile.mkdtemp()
    t = time.time()
    s = P.Scene(synthetic.diffuse_scene(d, ntri=1_000_000))
    s.build()
    print("1m build", time.time() - t, flush=True)
    cfg = P.RenderConfig(width=1280, height=1024, iterations=1, max_bounces=8)
    a, _ = t_gpu(s, cfg, "1m")
    o = t_oracle(s, cfg, "1m")
    print("equal", np.array_equal(a.view(np.uint32), o.view(np.uint32)), flush=True)
