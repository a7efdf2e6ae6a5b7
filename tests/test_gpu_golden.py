"""Full-size parity on the GPU: the reference's own configuration
(Scene.cpp scene, 1000x800, ITER = 500, 5 bounces).

* grid accel (the reference algorithm): the BMP payload must equal the
  committed 500-iteration oracle payload byte for byte, and therefore sit
  within the oracle's pinned distance of PathTracerAP/Render.bmp;
* BVH accel (exact closest hit): compared with Render.bmp under the same
  statistical bounds (it differs from the grid only where the grid's early
  exit misses a nearer triangle).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, REF_SCENE

pytestmark = pytest.mark.gpu


def _render_bmp_payload(P, accel, tmp_path):
    s = P.Scene(REF_SCENE)
    s.build(bvh=accel != 0)
    cfg = s.apply_settings(P.RenderConfig())
    cfg.accel = accel
    assert (cfg.width, cfg.height, cfg.iterations, cfg.max_bounces) == (1000, 800, 500, 5)
    r = P.Renderer(cfg)
    r.allocateOnGPU(s)
    r.renderLoop()
    out = tmp_path / f"Render_{accel}.bmp"
    r.renderImage(str(out))
    seg = r.segments()
    r.free()
    raw = out.read_bytes()
    assert len(raw) == 54 + 3 * 1000 * 800
    return np.frombuffer(raw[54:], np.uint8).reshape(800, 1000, 3), seg


def _stats(a, b):
    d = np.abs(a.astype(np.int32) - b.astype(np.int32))
    return (d == 0).mean(), (d <= 1).mean(), (d <= 2).mean(), d.max()


@pytest.mark.parametrize("accel", [0, 2])
def test_grid_full_size_equals_oracle_and_reference(gpu, pt_mod, tmp_path, accel):
    px, seg = _render_bmp_payload(pt_mod, accel, tmp_path)
    oracle_px = np.load(os.path.join(GOLDEN, "oracle_render_1000x800_500.npz"))["bgr"]
    assert seg == 1293177856
    assert np.array_equal(px, oracle_px), "GPU 500-iteration render differs from the pinned oracle render"
    ref = np.load(os.path.join(GOLDEN, "reference_render_1000x800_500.npz"))["bgr"]
    exact, w1, w2, mx = _stats(px, ref)
    assert exact > 0.75 and w1 > 0.99 and w2 > 0.9995 and mx <= 8


def test_bvh_full_size_vs_reference(gpu, pt_mod, tmp_path):
    """BVH = exact closest hit.  The reference grid disagrees on ~0.3% of rays
    (its entry-point check rejects rays whose rounded entry lands just outside
    a box's min faces; its DDA stops 3 voxels past the last hit voxel), and a
    single disagreement renumbers the compacted ray slots and so every later
    RNG seed of that iteration: the per-pixel noise decorrelates.  The image
    must agree statistically: per-channel means and 20x20-pixel block means."""
    px, _ = _render_bmp_payload(pt_mod, 1, tmp_path)
    ref = np.load(os.path.join(GOLDEN, "reference_render_1000x800_500.npz"))["bgr"]
    a, b = px.astype(np.float64), ref.astype(np.float64)
    mean_diff = np.abs(a.reshape(-1, 3).mean(0) - b.reshape(-1, 3).mean(0)).max()
    blk = lambda x: x.reshape(40, 20, 50, 20, 3).mean(axis=(1, 3))
    block_diff = np.abs(blk(a) - blk(b))
    print("bvh vs Render.bmp: mean diff", mean_diff, "block mean abs", block_diff.mean(), "block max", block_diff.max())
    assert mean_diff < 1.0
    assert block_diff.mean() < 1.5
    assert np.percentile(block_diff, 99) < 8.0
