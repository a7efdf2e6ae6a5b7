"""GPU parity at the iteration ids the bench's full-spp runs publish.

Every other oracle comparison renders iterations starting at 0.  The full
runs behind the bench line go up to id 255 (configs[1], 256 spp), 1023 (the
1M target and configs[2], 1024 spp) and 4095 (configs[4], 4096 spp), and the
per-ray seed is utilHash((1 << 31) | (depth << 22) | iter) ^ utilHash(slot)
(utility.h:58-62, with depth = remaining bounces up to 16).  These tests
render windows of those frames at exactly those ids, through
renderLoop(first_iter, n) (Renderer.cpp:567-648's `iter` argument), and
compare image and segment count with the oracle at the same first_iter, bit
for bit.  A window is the full frame's camera restricted by plane_x0/plane_y0
at the frame's own pixel pitch, so its rays are the full frame's rays; the
slot index (the seed's second input) is the window's own dense slot, as for
any frame size.
"""
import numpy as np
import pytest

from conftest import REF_SCENE
from helpers import assert_bitexact, flat_from_export, oracle_cfg

pytestmark = pytest.mark.gpu

THREADS = 16


@pytest.fixture(scope="module")
def synth_dir(tmp_path_factory):
    return str(tmp_path_factory.mktemp("iterscenes"))


def _window_cfg(P, width, height, x0, y0, side, bounces, pitch_w=20.0):
    step = pitch_w / width
    return P.RenderConfig(width=side, height=side, iterations=1, max_bounces=bounces,
                          plane_x0=-10.0 + x0 * step, plane_y0=-4.0 + y0 * step,
                          plane_w=side * step, plane_h=side * step)


def _both(P, O, scene, cfg, first_iter, n_iters):
    r = P.Renderer(cfg)
    r.allocateOnGPU(scene)
    r.renderLoop(first_iter, n_iters)
    img, seg, faults = r.image(), r.segments(), r.trace_faults()
    r.free()
    oc = oracle_cfg(cfg, threads=THREADS)
    oc.first_iter, oc.iterations = first_iter, n_iters
    oimg, oseg = O.render(flat_from_export(scene.export(), cfg.grid), oc)
    assert faults == 0
    return img, seg, oimg, oseg


def test_configs1_last_iterations_bitexact(gpu, pt_mod, oracle_mod, synth_dir):
    """configs[1] (~100k triangles, 8 bounces): ids 254 and 255, the last two of
    the 256-spp run, on a 128x128 window of the 1280x1024 frame."""
    from pathtracerap_amd import synthetic
    P, O = pt_mod, oracle_mod
    s = P.Scene(synthetic.diffuse_scene(synth_dir, ntri=100_000))
    s.build()
    cfg = _window_cfg(P, 1280, 1024, 576, 448, 128, 8)
    img, seg, oimg, oseg = _both(P, O, s, cfg, 254, 2)
    assert seg == oseg
    assert_bitexact(img, oimg, "configs[1] ids 254-255")


def test_target_1m_iteration_1023_bitexact(gpu, pt_mod, oracle_mod, synth_dir):
    """north_star target (1M triangles, 8 bounces): id 1023, the last of the
    1024-spp run, on a 64x64 window on the torus."""
    from pathtracerap_amd import synthetic
    P, O = pt_mod, oracle_mod
    s = P.Scene(synthetic.diffuse_scene(synth_dir, ntri=1_000_000))
    s.build()
    cfg = _window_cfg(P, 1280, 1024, 896, 432, 64, 8)
    img, seg, oimg, oseg = _both(P, O, s, cfg, 1023, 1)
    assert seg == oseg
    assert_bitexact(img, oimg, "1M target id 1023")


def test_configs2_iteration_1023_bitexact(gpu, pt_mod, oracle_mod):
    """configs[2] (the README scene, 5 bounces, metal and coat): ids 1022 and
    1023 on a 128x128 window of the 2800x2240 frame."""
    P, O = pt_mod, oracle_mod
    s = P.Scene(REF_SCENE)
    s.build()
    cfg = s.apply_settings(P.RenderConfig())
    assert cfg.max_bounces == 5
    w = _window_cfg(P, 2800, 2240, 1200, 900, 128, 5)
    w.grid = cfg.grid
    img, seg, oimg, oseg = _both(P, O, s, w, 1022, 2)
    assert seg == oseg
    assert_bitexact(img, oimg, "configs[2] ids 1022-1023")


@pytest.fixture(scope="module")
def scene_10m(pt_mod):
    from pathtracerap_amd import synthetic
    return synthetic.build_scene(pt_mod, ntri=10_000_000)


def test_configs4_iteration_4095_bitexact(gpu, pt_mod, oracle_mod, scene_10m):
    """configs[4] (10M triangles, 16 bounces): id 4095, the last of the
    4096-spp run, on the torus-face window of test_gpu_configs (the seed's
    depth field reaches 16 there)."""
    P, O = pt_mod, oracle_mod
    cfg = _window_cfg(P, 1280, 1024, 960, 416, 64, 16)
    img, seg, oimg, oseg = _both(P, O, scene_10m, cfg, 4095, 1)
    assert seg == oseg
    assert_bitexact(img, oimg, "configs[4] id 4095")
    assert np.isfinite(img).all() and img.sum() > 0


def test_configs1_full_frame_last_six_iterations_bitexact(gpu, pt_mod, oracle_mod, synth_dir):
    """configs[1] at full size (1280x1024, 8 bounces, the default 16 pipelines):
    ids 250..255, the last six of the 256-spp run, whole frame, against the
    oracle's render of the same ids -- with test_configs1_bench_workload_bitexact
    (ids 0-1) eight of the run's 256 iterations are pinned at full size."""
    from pathtracerap_amd import synthetic
    P, O = pt_mod, oracle_mod
    s = P.Scene(synthetic.diffuse_scene(synth_dir, ntri=100_000))
    s.build()
    cfg = P.RenderConfig(width=1280, height=1024, iterations=6, max_bounces=8)
    img, seg, oimg, oseg = _both(P, O, s, cfg, 250, 6)
    assert seg == oseg
    assert_bitexact(img, oimg, "configs[1] full frame ids 250-255")


def test_target_1m_full_frame_last_iterations_bitexact(gpu, pt_mod, oracle_mod, synth_dir):
    """north_star target (1M triangles) at full size: ids 1021..1023, the last
    three of the 1024-spp run, whole frame."""
    from pathtracerap_amd import synthetic
    P, O = pt_mod, oracle_mod
    s = P.Scene(synthetic.diffuse_scene(synth_dir, ntri=1_000_000))
    s.build()
    cfg = P.RenderConfig(width=1280, height=1024, iterations=3, max_bounces=8)
    img, seg, oimg, oseg = _both(P, O, s, cfg, 1021, 3)
    assert seg == oseg
    assert_bitexact(img, oimg, "1M target full frame ids 1021-1023")
