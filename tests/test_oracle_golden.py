"""Oracle pinning against the reference's own output image.

PathTracerAP/Render.bmp (1000x800, ITER=500, Scene.cpp scene) is the only
golden output the reference ships.  tests/golden/pin_oracle.py rendered the
same scene with the oracle (30 min on one core) and committed the BMP payload
(oracle_render_1000x800_500.npz) and the comparison statistics; these tests
re-derive the statistics from the two committed payloads and re-render a
cheap slice to check the committed payload still comes from this oracle.
"""
import json
import os

import numpy as np

from conftest import GOLDEN, INPUT_DATA


def _load():
    ref = np.load(os.path.join(GOLDEN, "reference_render_1000x800_500.npz"))["bgr"]
    ours = np.load(os.path.join(GOLDEN, "oracle_render_1000x800_500.npz"))["bgr"]
    return ref, ours


def test_oracle_matches_reference_render_bmp():
    ref, ours = _load()
    d = np.abs(ours.astype(np.int32) - ref.astype(np.int32))
    # thresholds: the CUDA build's FMA contraction / sinf ulps flip a few Monte-Carlo paths
    assert (d == 0).mean() > 0.75
    assert (d <= 1).mean() > 0.99
    assert (d <= 2).mean() > 0.9995
    assert d.max() <= 8
    assert d.mean() < 0.3
    st = json.load(open(os.path.join(GOLDEN, "oracle_pin_stats.json")))
    assert abs(st["mean_abs_diff"] - d.mean()) < 1e-9
    assert st["segments"] == 1293177856


def test_reference_header_layout():
    hdr = np.load(os.path.join(GOLDEN, "reference_render_1000x800_500.npz"))["header"].tobytes()
    import oracle as O
    mine = O.to_bmp_bytes(np.zeros((1000 * 800, 3), np.float32), 1000, 800, 500)[:54]
    assert hdr == mine, "Renderer::renderImage header layout"


def test_committed_payload_is_this_oracle(oracle_mod):
    """Two full-resolution oracle iterations: the per-channel mean and a
    coarse block structure must agree with the committed 500-iteration
    payload (the 500-iteration render itself is too slow for CI)."""
    ref, ours = _load()
    sc = oracle_mod.reference_scene(INPUT_DATA)
    img, _ = oracle_mod.render(sc, oracle_mod.RenderConfig(width=1000, height=800, iterations=2, threads=0))
    px = np.frombuffer(oracle_mod.to_bmp_bytes(img, 1000, 800, 2)[54:], np.uint8).reshape(800, 1000, 3)
    assert np.abs(px.reshape(-1, 3).mean(0) - ours.reshape(-1, 3).mean(0)).max() < 1.5
    blk = lambda a: a.astype(np.float64).reshape(16, 50, 20, 50, 3).mean(axis=(1, 3))
    assert np.abs(blk(px) - blk(ours)).mean() < 4.0
