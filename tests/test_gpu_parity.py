"""GPU parity: the HIP path (through the C ABI) vs the CPU oracle.

Bar: bit-exact.  Every float the kernels produce follows the reference's
operation order (no contraction), the RNG is the reference's hash + minstd,
and the compaction reproduces thrust::stable_partition's slot order, so the
accumulated image must match the oracle bit for bit.
"""
import numpy as np
import pytest

from conftest import REF_SCENE
from helpers import assert_bitexact, flat_from_export, oracle_cfg

pytestmark = pytest.mark.gpu


def _ref_scene(P, bvh=False):
    s = P.Scene(REF_SCENE)
    s.build(bvh=bvh)
    return s


@pytest.mark.parametrize("accel", [0, 1, 2])
def test_primary_hits_bitexact(gpu, pt_mod, oracle_mod, accel):
    P, O = pt_mod, oracle_mod
    s = _ref_scene(P, bvh=accel != 0)
    cfg = P.RenderConfig(width=160, height=128, iterations=1, accel=accel)
    r = P.Renderer(cfg)
    r.allocateOnGPU(s)
    d, n, m = r.primary_hits()
    r.free()
    od, on, om = O.intersect_primary(flat_from_export(s.export()), oracle_cfg(cfg))
    assert_bitexact(m, om, "model")
    assert_bitexact(d, od, "dist")
    hit = om >= 0
    assert_bitexact(n[hit], on[hit], "normal")


@pytest.mark.parametrize("accel", [0, 1, 2])
def test_render_reference_scene_bitexact(gpu, pt_mod, oracle_mod, accel):
    P, O = pt_mod, oracle_mod
    s = _ref_scene(P, bvh=accel != 0)
    cfg = P.RenderConfig(width=200, height=160, iterations=3, accel=accel)
    r = P.Renderer(cfg)
    r.allocateOnGPU(s)
    r.renderLoop()
    img = r.image()
    seg = r.segments()
    r.free()
    oimg, oseg = O.render(flat_from_export(s.export()), oracle_cfg(cfg))
    assert seg == oseg
    assert_bitexact(img, oimg, "image")


def test_grid_only_scene_shared_by_three_renderers(gpu, pt_mod, oracle_mod):
    """A scene built grid-only (build(bvh=False)) and shared by renderers of all three
    modes, allocated from three threads at once (ctypes drops the GIL): the first
    grid_fast / bvh allocation adds the BLAS under the scene's lock
    (capi.cpp pt_renderer_allocate_on_gpu), and every image still equals the oracle's."""
    from concurrent.futures import ThreadPoolExecutor
    P, O = pt_mod, oracle_mod
    s = _ref_scene(P, bvh=False)
    rs = [P.Renderer(P.RenderConfig(width=160, height=128, iterations=2, accel=a)) for a in (2, 1, 0)]
    with ThreadPoolExecutor(3) as ex:
        list(ex.map(lambda r: r.allocateOnGPU(s), rs))
    flat = flat_from_export(s.export())
    for r in rs:
        r.renderLoop()
        img, seg = r.image(), r.segments()
        oimg, oseg = O.render(flat, oracle_cfg(r.cfg))
        r.free()
        assert seg == oseg
        assert_bitexact(img, oimg, "image")
