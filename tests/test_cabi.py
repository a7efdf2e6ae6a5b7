"""The C-ABI library loads and exports every symbol include/pathtracer_amd.h
declares (no compute calls: runs without a GPU)."""
import ctypes
import os
import re

from conftest import ROOT


def _declared():
    txt = open(os.path.join(ROOT, "include", "pathtracer_amd.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pt_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol(pt_mod):
    L = ctypes.CDLL(os.path.join(ROOT, "pathtracerap_amd", "libpathtracer_amd.so"))
    names = _declared()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    bound = {n for n, _, _ in pt_mod.EXPORTS}
    assert set(names) == bound, set(names) ^ bound


def test_abi_version_and_defaults(pt_mod):
    L = pt_mod.lib()
    assert L.pt_abi_version() == 8
    c = pt_mod._Cfg()
    L.pt_default_config(ctypes.byref(c))
    # Config.h / generateRaysKernel defaults
    assert (c.width, c.height, c.iterations, c.max_bounces) == (1000, 800, 500, 5)
    assert tuple(c.grid) == (25, 25, 25) and tuple(c.cam) == (0.0, 0.0, 920.0)
    assert (c.plane_x0, c.plane_y0, c.plane_w, c.plane_h, c.plane_z) == (-10.0, -4.0, 20.0, 16.0, 900.0)
    # the drop-in default is the fast path with the reference's results: grid_fast
    assert c.accel == pt_mod.ACCEL_GRID_FAST
    # throughput knobs (results identical for every value): the struct tail matches the header
    assert (c.block, c.pipelines, c.ray_sort) == (64, 16, -1)
    py = pt_mod.RenderConfig()
    assert (py.accel, py.block, py.pipelines, py.ray_sort) == (c.accel, c.block, c.pipelines, c.ray_sort)


def test_library_load_sets_hw_queues_unless_chosen():
    """Loading libpathtracer_amd.so gives the process one hardware queue per
    pipeline stream (GPU_MAX_HW_QUEUES=16) unless the variable is already set."""
    import subprocess
    import sys
    code = ("import ctypes; ctypes.CDLL(%r); libc = ctypes.CDLL(None); libc.getenv.restype = ctypes.c_char_p; "
            "print(libc.getenv(b'GPU_MAX_HW_QUEUES'))") % os.path.join(ROOT, "pathtracerap_amd", "libpathtracer_amd.so")
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True).stdout
    assert out.strip() == "b'16'"
    env["GPU_MAX_HW_QUEUES"] = "4"
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True).stdout
    assert out.strip() == "b'4'"


def test_hw_queue_info_reports_the_setting_found_at_load():
    """pt_hw_queue_info / hw_queues(): the value the process had chosen (or that
    the library set 16)."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import pathtracerap_amd as P; q = P.hw_queues(); "
            "print(P._lib is not None, q)") % ROOT
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True).stdout
    assert out.startswith("True ") and "'at_library_load': None, 'set_by_library': True, 'env_now': 16" in out, out
    env["GPU_MAX_HW_QUEUES"] = "4"
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True).stdout
    assert "'at_library_load': 4, 'set_by_library': False, 'env_now': 4" in out, out


def test_errors_are_reported_not_crashing(pt_mod):
    L = pt_mod.lib()
    assert L.pt_scene_load_config(None, b"x") == -1
    assert b"null scene" in L.pt_last_error()
    assert L.pt_renderer_render_loop(None, 0, 1) == -1
    c = pt_mod._Cfg()
    L.pt_default_config(ctypes.byref(c))
    c.accel = 7
    assert L.pt_renderer_create(ctypes.byref(c)) is None
    assert b"bad accel" in L.pt_last_error()


def test_renderer_requires_built_scene(pt_mod):
    s = pt_mod.Scene()
    r = pt_mod.Renderer(pt_mod.RenderConfig(width=8, height=8))
    try:
        import pytest
        with pytest.raises(pt_mod.PathTracerError, match="not built"):
            r.allocateOnGPU(s)
    finally:
        r.free()
