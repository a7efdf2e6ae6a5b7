"""GPU parity at the BASELINE.json configurations' own sizes (the reference's
bounce loop, Renderer.cpp:567-648, against the CPU oracle, bit for bit).

* configs[1]: the ~100k-triangle diffuse synthetic scene, 1280x1024, 8 bounces,
  2 iterations -- the bench workload itself, through the drop-in defaults
  (grid_fast, 16 pipelines, ray sort, drain continuations, walk hand-ons);
* north_star target: the 1M-triangle scene, 1280x1024, 8 bounces, 1 iteration;
* configs[2]: the README render's scene (Scene.cpp:3-224 =
  scenes/reference_scene.txt) at 2800x2240, 5 bounces, 1 iteration;
* configs[4]: the 10M-triangle scene, 16 bounces (deep BLAS at the depth cap,
  dense hit sets): five disjoint 64x64 windows of the frame against the oracle
  (torus face, silhouette, back wall, floor under the lamp, ring's inner face),
  plus full-frame properties (no trace faults, finite image, per-bounce ray
  counts);
* the drop-in entry points with no configuration: pt_render (main.cpp:11-27)
  and the pathtracer_amd CLI render the reference scene at its own settings
  (1000x800, ITER 500) byte-identical to the committed oracle render.

The oracle runs on 16 host threads; every case finishes in well under a minute
on the GPU box.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, REF_SCENE, ROOT
from helpers import assert_bitexact, flat_from_export, oracle_cfg

pytestmark = pytest.mark.gpu

THREADS = 16


@pytest.fixture(scope="module")
def synth_dir(tmp_path_factory):
    return str(tmp_path_factory.mktemp("cfgscenes"))


def _gpu_render(P, scene, cfg):
    r = P.Renderer(cfg)
    r.allocateOnGPU(scene)
    r.renderLoop()
    out = dict(img=r.image(), seg=r.segments(), per_bounce=r.segments_per_bounce(cfg.max_bounces + 1),
               faults=r.trace_faults(), pipes=r.pipelines())
    r.free()
    return out


def _oracle_render(O, scene, cfg):
    img, seg = O.render(flat_from_export(scene.export(), cfg.grid), oracle_cfg(cfg, threads=THREADS))
    return img, seg


def test_configs1_bench_workload_bitexact(gpu, pt_mod, oracle_mod, synth_dir):
    """configs[1] at full size through the defaults the bench and the drop-in use."""
    from pathtracerap_amd import synthetic
    P, O = pt_mod, oracle_mod
    s = P.Scene(synthetic.diffuse_scene(synth_dir, ntri=100_000))
    s.build()
    assert s.counts()["nt"] > 99_000
    cfg = s.apply_settings(P.RenderConfig())
    cfg.iterations = 2
    assert (cfg.width, cfg.height, cfg.max_bounces) == (1280, 1024, 8)
    assert cfg.accel == P.ACCEL_GRID_FAST and cfg.pipelines == 16
    g = _gpu_render(P, s, cfg)
    assert g["pipes"] == 16 and g["faults"] == 0
    oimg, oseg = _oracle_render(O, s, cfg)
    assert g["seg"] == oseg
    assert_bitexact(g["img"], oimg, "configs[1] 1280x1024 image")


def test_target_1m_triangles_bitexact(gpu, pt_mod, oracle_mod, synth_dir):
    """north_star target scene (1M-triangle diffuse OBJ) at 1280x1024."""
    from pathtracerap_amd import synthetic
    P, O = pt_mod, oracle_mod
    s = P.Scene(synthetic.diffuse_scene(synth_dir, ntri=1_000_000))
    s.build()
    assert s.counts()["nt"] > 990_000
    cfg = P.RenderConfig(width=1280, height=1024, iterations=1, max_bounces=8)
    g = _gpu_render(P, s, cfg)
    assert g["faults"] == 0
    oimg, oseg = _oracle_render(O, s, cfg)
    assert g["seg"] == oseg
    assert_bitexact(g["img"], oimg, "1M-triangle 1280x1024 image")


@pytest.mark.parametrize("ntri,side", [(100_000, 48), (1_000_000, 16)])
def test_bvh_mode_window_bitexact_at_size(gpu, pt_mod, oracle_mod, synth_dir, ntri, side):
    """The exact-closest-hit mode (PT_ACCEL_BVH, bench alt_mode) at the configs[1]
    and target scene sizes: a window of the 1280x1024 frame on the torus against
    the oracle's exhaustive closest hit over every triangle (accel = 1)."""
    from pathtracerap_amd import synthetic
    P, O = pt_mod, oracle_mod
    s = P.Scene(synthetic.diffuse_scene(synth_dir, ntri=ntri))
    s.build()
    step = 20.0 / 1280                                 # the full frame's pixel pitch (exact in binary)
    cfg = P.RenderConfig(width=side, height=side, iterations=1, max_bounces=8, accel=P.ACCEL_BVH,
                         plane_x0=-10.0 + 896 * step, plane_y0=-4.0 + 432 * step,
                         plane_w=side * step, plane_h=side * step)
    g = _gpu_render(P, s, cfg)
    assert g["faults"] == 0
    oimg, oseg = _oracle_render(O, s, cfg)
    assert g["seg"] == oseg
    assert_bitexact(g["img"], oimg, f"bvh mode, {ntri} triangles")


def test_configs2_readme_scene_2800x2240_bitexact(gpu, pt_mod, oracle_mod):
    """configs[2]: the README render's own scene (metal, coat, diffuse and
    emissive models of Scene.cpp) at 2800x2240, the reference's 5 bounces."""
    P, O = pt_mod, oracle_mod
    s = P.Scene(REF_SCENE)
    s.build()
    cfg = s.apply_settings(P.RenderConfig())
    cfg.width, cfg.height, cfg.iterations = 2800, 2240, 1
    assert cfg.max_bounces == 5
    g = _gpu_render(P, s, cfg)
    assert g["faults"] == 0
    oimg, oseg = _oracle_render(O, s, cfg)
    assert g["seg"] == oseg
    assert_bitexact(g["img"], oimg, "configs[2] 2800x2240 image")


@pytest.fixture(scope="module")
def scene_10m(pt_mod):
    from pathtracerap_amd import synthetic
    return synthetic.build_scene(pt_mod, ntri=10_000_000)


def _bvh_depth(scene):
    """Deepest level of the binary BLAS (root = 1), by a vectorised walk."""
    b = scene.export_bvh()
    nodes = b["nodes"].view(np.int32)
    depth, frontier = 0, np.unique(b["roots"][b["roots"] >= 0])
    while len(frontier):
        depth += 1
        n = nodes[frontier]
        # BvhNode: (lo0.xyz, link0) (hi0.xyz, link1) (lo1.xyz, cnt0) (hi1.xyz, cnt1); cnt 0 = inner child
        link = np.stack([n[:, 3], n[:, 7]], 1)
        cnt = np.stack([n[:, 11], n[:, 15]], 1)
        frontier = link[cnt == 0]
    return depth


# 64x64 windows of the configs[4] frame, full-frame pixel origin (x0, y0) at the
# frame's own pixel pitch 20/1280 (exact in binary), and the model the window's
# primary rays must mostly see (1 = the 10M-triangle torus, 0 = the room)
CONFIGS4_WINDOWS = {
    "torus_ring_face": ((960, 416), 1),
    "torus_silhouette": ((384, 608), None),       # ring edge against the back wall: both models
    "back_wall": ((800, 800), 0),
    "floor_under_light": ((640, 0), 0),
    "ring_inner_face": ((448, 384), None),        # the hole: inner face and the wall seen through it
}


@pytest.mark.parametrize("window", sorted(CONFIGS4_WINDOWS))
def test_configs4_10m_triangles_window_bitexact(gpu, pt_mod, oracle_mod, scene_10m, window):
    """configs[4]: 10M triangles, 16 bounces -- five disjoint 64x64 windows of
    the 1280x1024 frame (plane_x0/plane_y0 select them) against the oracle, bit
    for bit: the torus ring's face, its silhouette against the wall, the back
    wall, the floor under the front lamp and the ring's inner face."""
    P, O = pt_mod, oracle_mod
    s = scene_10m
    assert s.counts()["nt"] > 9_900_000
    assert _bvh_depth(s) <= 24          # bvh.cpp kMaxDepth = 23 holds at 10M triangles (node levels incl. the root)
    (x0, y0), dominant = CONFIGS4_WINDOWS[window]
    step = 20.0 / 1280
    cfg = P.RenderConfig(width=64, height=64, iterations=1, max_bounces=16,
                         plane_x0=-10.0 + x0 * step, plane_y0=-4.0 + y0 * step, plane_w=64 * step, plane_h=64 * step)
    g = _gpu_render(P, s, cfg)
    assert g["faults"] == 0
    oimg, oseg = _oracle_render(O, s, cfg)
    assert g["seg"] == oseg
    assert_bitexact(g["img"], oimg, f"configs[4] 10M-triangle window {window}")
    r = P.Renderer(cfg)
    r.allocateOnGPU(s)
    _, _, m = r.primary_hits()
    r.free()
    if dominant is None:
        assert (m == 0).mean() > 0.1 and (m == 1).mean() > 0.1
    else:
        assert (m == dominant).mean() > 0.5


def test_configs4_10m_triangles_full_frame_properties(gpu, pt_mod, scene_10m):
    """configs[4] full frame (1280x1024, 16 bounces): no trace faults, a finite
    image, rays reaching deep bounces, and every bounce's ray count consistent
    with the segment total (the windows above are the oracle check)."""
    P = pt_mod
    s = scene_10m
    cfg = P.RenderConfig(width=1280, height=1024, iterations=1, max_bounces=16)
    g = _gpu_render(P, s, cfg)
    assert g["faults"] == 0
    assert np.isfinite(g["img"]).all() and g["img"].sum() > 0
    pb = g["per_bounce"]
    assert pb[0] == 1280 * 1024 and pb[8] > 0 and sum(pb) == g["seg"]
    assert all(a >= b for a, b in zip(pb, pb[1:]))          # compaction only removes rays


def _oracle_bmp_payload():
    return np.load(os.path.join(GOLDEN, "oracle_render_1000x800_500.npz"))["bgr"]


def _bmp_payload(path):
    raw = open(path, "rb").read()
    assert len(raw) == 54 + 3 * 1000 * 800
    return np.frombuffer(raw[54:], np.uint8).reshape(800, 1000, 3)


def test_pt_render_defaults_equal_oracle(gpu, pt_mod, tmp_path):
    """pt_render (main.cpp:11-27) with no configuration: the reference scene at
    its own settings through the default path (grid_fast, 16 pipelines) writes
    the oracle's 500-iteration Render.bmp byte for byte."""
    out = tmp_path / "Render.bmp"
    pt_mod.render(REF_SCENE, None, str(out))
    assert np.array_equal(_bmp_payload(out), _oracle_bmp_payload())


def test_cli_defaults_equal_oracle(gpu, pt_mod, tmp_path):
    """The pathtracer_amd CLI with no flags: same bytes."""
    exe = os.path.join(ROOT, "pathtracerap_amd", "pathtracer_amd")
    out = tmp_path / "Render.bmp"
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    p = subprocess.run([exe, REF_SCENE, str(out)], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr
    assert "Mrays/s" in p.stdout
    assert np.array_equal(_bmp_payload(out), _oracle_bmp_payload())


def test_configs4_10m_triangles_320x256_grid_fast_equals_grid(gpu, pt_mod, scene_10m):
    """configs[4]'s view on a whole 320x256 frame, 16 bounces: the benched
    grid_fast path (4-wide node steps, ray sort, sparse-bounce launch sizing,
    drain and walk hand-ons) against the reference grid mode (the list-walking
    DDA, the literal restatement of Renderer.cpp:238-360), image and every
    bounce's live-ray count bit for bit -- whole-frame coverage beside the
    five oracle windows."""
    P = pt_mod
    small = P.RenderConfig(width=320, height=256, iterations=1, max_bounces=16)
    a = _gpu_render(P, scene_10m, small)
    small.accel = P.ACCEL_GRID
    b = _gpu_render(P, scene_10m, small)
    assert a["faults"] == 0 and b["faults"] == 0
    assert a["per_bounce"] == b["per_bounce"]
    assert_bitexact(a["img"], b["img"], "grid_fast vs grid, 10M triangles, 320x256")
