"""configs[0] as BASELINE.json states it: the Cornell-box scene from the
reference's Input data/ (Scene.cpp:3-224 over enclosing_box / ceiling_light /
blender_monkey .obj), 256x256, 4 samples per pixel, the reference's 5 bounces
(Renderer.cpp:550), on the serial CPU loop (the oracle with threads = 1;
Renderer.cpp:567-648) -- and the HIP path at the same config, bit for bit.

Parity basis: the HIP path is bit-exact against the C restatement
(oracle/ptoracle.c); the restatement is within 1 LSB of the reference's
Render.bmp on 99.4 % of channels (max 4; tests/test_oracle_golden.py).  Here the
4-spp render's 4x4 / 8x8 block means are also held to Render.bmp's (500 spp).
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, INPUT_DATA, REF_SCENE
from helpers import assert_bitexact, flat_from_export, oracle_cfg

W, H, SPP, BOUNCES = 256, 256, 4, 5


def _fixture():
    with open(os.path.join(GOLDEN, "configs0_256x256_4spp.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def serial_render(oracle_mod):
    O = oracle_mod
    sc = O.reference_scene(INPUT_DATA)
    img, seg = O.render(sc, O.RenderConfig(width=W, height=H, iterations=SPP, max_bounces=BOUNCES, threads=1))
    return img, seg


def test_configs0_serial_loop_matches_fixture(oracle_mod, serial_render):
    img, seg = serial_render
    fx = _fixture()
    assert (fx["width"], fx["height"], fx["spp"], fx["max_bounces"], fx["threads"]) == (W, H, SPP, BOUNCES, 1)
    assert seg == fx["segments"]
    assert hashlib.sha256(img.tobytes()).hexdigest() == fx["image_sha256"]
    assert hashlib.sha256(oracle_mod.to_bmp_bytes(img, W, H, SPP)).hexdigest() == fx["bmp_sha256"]
    assert np.isfinite(img).all()


def test_configs0_serial_equals_threaded(oracle_mod, serial_render):
    """The serial loop and the OpenMP one trace the same rays in the same order
    per pixel: identical images (every ray's RNG seed is fixed by its slot)."""
    O = oracle_mod
    img1, seg1 = serial_render
    sc = O.reference_scene(INPUT_DATA)
    img8, seg8 = O.render(sc, O.RenderConfig(width=W, height=H, iterations=SPP, max_bounces=BOUNCES, threads=8))
    assert seg8 == seg1
    assert np.array_equal(img8.view(np.uint32), img1.view(np.uint32))


def test_configs0_block_means_match_reference_render_bmp(oracle_mod, serial_render):
    """The same view as the reference's Render.bmp (1000x800, 500 spp): block
    means over the 4 x 4 and 8 x 8 tilings of the image plane agree within a
    few 8-bit levels (4-spp Monte-Carlo noise)."""
    img, _ = serial_render
    px = np.frombuffer(oracle_mod.to_bmp_bytes(img, W, H, SPP)[54:], np.uint8).reshape(H, W, 3).astype(np.float64)
    ref = np.load(os.path.join(GOLDEN, "reference_render_1000x800_500.npz"))["bgr"].astype(np.float64)
    for nb, tol_max, tol_mean in ((4, 3.0, 1.2), (8, 6.0, 2.0)):
        a = px.reshape(nb, H // nb, nb, W // nb, 3).mean(axis=(1, 3))
        b = ref.reshape(nb, 800 // nb, nb, 1000 // nb, 3).mean(axis=(1, 3))
        d = np.abs(a - b)
        assert d.max() < tol_max and d.mean() < tol_mean, (nb, d.max(), d.mean())


def test_configs0_product_loader_scene_is_the_reference_scene(pt_mod, oracle_mod, serial_render):
    """The drop-in loader (scenes/reference_scene.txt in the Config.txt grammar)
    builds the scene the oracle builds from Scene.cpp: same serial render."""
    P, O = pt_mod, oracle_mod
    img1, seg1 = serial_render
    s = P.Scene(REF_SCENE)
    s.build()
    want, wseg = O.render(flat_from_export(s.export()), oracle_cfg(
        P.RenderConfig(width=W, height=H, iterations=SPP, max_bounces=BOUNCES), threads=1))
    assert wseg == seg1 and np.array_equal(want.view(np.uint32), img1.view(np.uint32))


@pytest.mark.gpu
def test_configs0_hip_path_bitexact(gpu, pt_mod, oracle_mod, serial_render):
    """The HIP path at configs[0] through the drop-in Scene loader: the default
    grid_fast mode and the literal grid mode render the serial loop's image bit
    for bit, and its segment count."""
    P, O = pt_mod, oracle_mod
    img1, seg1 = serial_render
    s = P.Scene(REF_SCENE)
    s.build()
    for accel in (P.ACCEL_GRID_FAST, P.ACCEL_GRID):
        cfg = P.RenderConfig(width=W, height=H, iterations=SPP, max_bounces=BOUNCES, accel=accel)
        r = P.Renderer(cfg)
        r.allocateOnGPU(s)
        r.renderLoop()
        got, seg, faults = r.image(), r.segments(), r.trace_faults()
        r.free()
        assert faults == 0 and seg == seg1
        assert_bitexact(got, img1, f"configs[0] accel={accel}")
