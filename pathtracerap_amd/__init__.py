"""MI355X-native PathTracerAP hot path.

Python mirror of the reference's host interface (Scene.h / Renderer.h of
purvakulkarni15/PathTracerAP) over the C ABI in ``include/pathtracer_amd.h``
(``libpathtracer_amd.so``: C++ host + gfx950 HIP kernels)::

    scene = Scene("scenes/reference_scene.txt")      # Scene::Scene(string config)
    renderer = Renderer(RenderConfig())              # Config.h constants at runtime
    renderer.allocateOnGPU(scene)                    # Renderer::allocateOnGPU
    renderer.renderLoop()                            # Renderer::renderLoop
    renderer.renderImage("Render.bmp")               # Renderer::renderImage
    renderer.free()                                  # Renderer::free

There is no CPU fallback: if the shared library is missing or no gfx950
device is present, the calls raise.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

__all__ = ["Scene", "Renderer", "RenderConfig", "PathTracerError", "build", "lib", "hw_queues",
           "MATERIALS", "ACCEL_GRID", "ACCEL_BVH", "ACCEL_GRID_FAST"]

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.environ.get("PT_LIB_PATH") or os.path.join(_HERE, "libpathtracer_amd.so")   # override: experiments

ACCEL_GRID = 0
ACCEL_BVH = 1
ACCEL_GRID_FAST = 2
# renderer.h: segments[] slots after the per-bounce counters, as segments_per_bounce indices
_MAX_BOUNCE_COUNTERS = 64
_DEFERRED_SLOT = 50 + _MAX_BOUNCE_COUNTERS - 1     # kDeferredRayCounter
# Primitive.h:70-79
MATERIALS = {"DIFFUSE": 0, "SPECULAR": 1, "REFLECTIVE": 2, "REFRACTIVE": 3,
             "EMISSIVE": 4, "COAT": 5, "METAL": 6}


class PathTracerError(RuntimeError):
    pass


def build(force: bool = False, jobs: int = 4) -> str:
    """Compile libpathtracer_amd.so for gfx950 in-tree (hipcc, no GPU needed)."""
    cmd = ["make", "-s", "-C", _HERE, f"-j{jobs}"]
    if force:
        subprocess.check_call(["make", "-s", "-C", _HERE, "clean"])
    subprocess.check_call(cmd)
    return _LIB_PATH


class _Cfg(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int), ("height", ctypes.c_int), ("iterations", ctypes.c_int),
        ("max_bounces", ctypes.c_int), ("accel", ctypes.c_int), ("grid", ctypes.c_int * 3),
        ("tail_drop", ctypes.c_int), ("cam", ctypes.c_double * 3), ("plane_z", ctypes.c_double),
        ("plane_x0", ctypes.c_double), ("plane_y0", ctypes.c_double),
        ("plane_w", ctypes.c_double), ("plane_h", ctypes.c_double), ("block", ctypes.c_int),
        ("pipelines", ctypes.c_int), ("ray_sort", ctypes.c_int),
    ]


_P_F = ctypes.POINTER(ctypes.c_float)
_P_I = ctypes.POINTER(ctypes.c_int)
_lib = None
_HIP_BEFORE_LOAD = None     # set when the library loads (torch's HIP runtime already up?)

# (name, restype, argtypes) of every exported symbol of include/pathtracer_amd.h
EXPORTS = [
    ("pt_abi_version", ctypes.c_int, []),
    ("pt_last_error", ctypes.c_char_p, []),
    ("pt_hw_queue_info", ctypes.c_int, [_P_I, _P_I]),
    ("pt_default_config", None, [ctypes.POINTER(_Cfg)]),
    ("pt_scene_create", ctypes.c_void_p, []),
    ("pt_scene_destroy", None, [ctypes.c_void_p]),
    ("pt_scene_load_config", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p]),
    ("pt_scene_apply_settings", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(_Cfg)]),
    ("pt_scene_load_obj", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p]),
    ("pt_scene_add_mesh", ctypes.c_int, [ctypes.c_void_p, _P_F, _P_F, ctypes.c_int, _P_I, ctypes.c_int]),
    ("pt_scene_add_model", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, _P_F, _P_F, _P_F, ctypes.c_int, _P_F]),
    ("pt_scene_build", ctypes.c_int, [ctypes.c_void_p, _P_I, ctypes.c_int]),
    ("pt_scene_counts", ctypes.c_int, [ctypes.c_void_p, _P_I]),
    ("pt_scene_export", ctypes.c_int, [ctypes.c_void_p, _P_F, _P_F, _P_I, _P_I, _P_F, _P_I, _P_F, _P_F,
                                       _P_F, _P_I, _P_F, _P_I, _P_I]),
    ("pt_scene_export_bvh", ctypes.c_int, [ctypes.c_void_p, _P_F, _P_I, _P_I]),
    ("pt_scene_export_bvh4", ctypes.c_int, [ctypes.c_void_p, _P_F, _P_I]),
    ("pt_scene_export_bvh4_leaf_base", ctypes.c_int, [ctypes.c_void_p, _P_I]),
    ("pt_renderer_create", ctypes.c_void_p, [ctypes.POINTER(_Cfg)]),
    ("pt_renderer_set_stream", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    ("pt_renderer_bind_image", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    ("pt_renderer_allocate_on_gpu", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    ("pt_renderer_clear_image", ctypes.c_int, [ctypes.c_void_p]),
    ("pt_renderer_render_loop", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    ("pt_renderer_synchronize", ctypes.c_int, [ctypes.c_void_p]),
    ("pt_renderer_read_image", ctypes.c_int, [ctypes.c_void_p, _P_F]),
    ("pt_renderer_render_image", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]),
    ("pt_renderer_segments", ctypes.c_longlong, [ctypes.c_void_p]),
    ("pt_renderer_trace_faults", ctypes.c_longlong, [ctypes.c_void_p]),
    ("pt_renderer_segments_per_bounce", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]),
    ("pt_renderer_pipelines", ctypes.c_int, [ctypes.c_void_p]),
    ("pt_renderer_set_profiling", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("pt_renderer_kernel_stats", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]),
    ("pt_renderer_kernel_stats_ex", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
    ("pt_renderer_primary_hits", ctypes.c_int, [ctypes.c_void_p, _P_F, _P_F, _P_I]),
    ("pt_renderer_intersect_rays", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, _P_F, _P_F, _P_F, _P_F, _P_I]),
    ("pt_renderer_certify_check", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, _P_F, _P_F, _P_I]),
    ("pt_renderer_free", None, [ctypes.c_void_p]),
    ("pt_selftest_math", ctypes.c_int, [ctypes.c_int, _P_F, _P_F, _P_F]),
    ("pt_render", ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(_Cfg), ctypes.c_char_p]),
]


def lib() -> ctypes.CDLL:
    """Load the in-tree HIP library; raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise PathTracerError(
                f"{_LIB_PATH} not found: run `make -C pathtracerap_amd` (or __graft_entry__.build())")
        global _HIP_BEFORE_LOAD
        import sys
        tc = sys.modules.get("torch.cuda")
        _HIP_BEFORE_LOAD = bool(tc is not None and tc.is_initialized())
        L = ctypes.CDLL(_LIB_PATH)
        for name, res, args in EXPORTS:
            if os.environ.get("PT_LIB_PATH") and not hasattr(L, name):
                continue            # an older build loaded for an A/B baseline: bind what it has
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def hw_queues() -> dict:
    """GPU_MAX_HW_QUEUES as the library found it at load (None: unset, then the
    library set 16), and whether HIP had already started in this process when the
    library loaded (then HIP runs with the value it read at its own start)."""
    a, s = ctypes.c_int(), ctypes.c_int()
    lib().pt_hw_queue_info(ctypes.byref(a), ctypes.byref(s))
    libc = ctypes.CDLL(None)            # the C environment (os.environ is a snapshot taken at start-up)
    libc.getenv.restype = ctypes.c_char_p
    env = libc.getenv(b"GPU_MAX_HW_QUEUES")
    env = env.decode() if env else None
    return {"at_library_load": None if a.value < 0 else a.value, "set_by_library": bool(s.value),
            "env_now": int(env) if env and env.isdigit() else None, "hip_started_before_load": _HIP_BEFORE_LOAD}


def _err(rc, what):
    if rc is None or (isinstance(rc, int) and rc < 0):
        msg = lib().pt_last_error()
        raise PathTracerError(f"{what}: {msg.decode() if msg else 'error'}")
    return rc


def _fp(a):
    return a.ctypes.data_as(_P_F)


def _ip(a):
    return a.ctypes.data_as(_P_I)


@dataclass
class RenderConfig:
    """Config.h (RESOLUTION_X/Y, ITER, GRID_X/Y/Z) and generateRaysKernel's
    constants (camera, image plane, bounce count), as runtime values."""
    width: int = 1000
    height: int = 800
    iterations: int = 500
    max_bounces: int = 5
    accel: int = ACCEL_GRID_FAST   # the reference grid's results, bit for bit (ACCEL_GRID: its list-walking DDA)
    grid: tuple = (25, 25, 25)
    tail_drop: int = 0
    cam: tuple = (0.0, 0.0, 920.0)
    plane_z: float = 900.0
    plane_x0: float = -10.0
    plane_y0: float = -4.0
    plane_w: float = 20.0
    plane_h: float = 16.0
    block: int = 64
    pipelines: int = 16   # iterations in flight (own HIP streams); results identical for any value
    ray_sort: int = -1    # ray sort key before each persistent trace (-1 auto, 0 off); results identical

    def c(self) -> _Cfg:
        c = _Cfg()
        c.width, c.height, c.iterations, c.max_bounces = self.width, self.height, self.iterations, self.max_bounces
        c.accel, c.tail_drop = self.accel, self.tail_drop
        for k in range(3):
            c.grid[k] = int(self.grid[k])
            c.cam[k] = float(self.cam[k])
        c.plane_z, c.plane_x0, c.plane_y0, c.plane_w, c.plane_h = (
            self.plane_z, self.plane_x0, self.plane_y0, self.plane_w, self.plane_h)
        c.block = self.block
        c.pipelines = self.pipelines
        c.ray_sort = self.ray_sort
        return c


class Scene:
    """Scene (Scene.h:21-40).  ``Scene(config_path)`` parses a Config.txt
    grammar file; ``Scene()`` starts empty for programmatic construction."""

    def __init__(self, config: str | None = None):
        self._h = lib().pt_scene_create()
        if not self._h:
            raise PathTracerError("pt_scene_create failed")
        if config is not None:
            _err(lib().pt_scene_load_config(self._h, os.fsencode(config)), f"load {config}")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.pt_scene_destroy(h)
            self._h = None

    def apply_settings(self, cfg: RenderConfig) -> RenderConfig:
        c = cfg.c()
        _err(lib().pt_scene_apply_settings(self._h, ctypes.byref(c)), "apply_settings")
        cfg.width, cfg.height, cfg.iterations, cfg.max_bounces, cfg.accel = (
            c.width, c.height, c.iterations, c.max_bounces, c.accel)
        cfg.grid = tuple(c.grid)
        return cfg

    def loadAndProcessMeshFile(self, path: str) -> int:
        return _err(lib().pt_scene_load_obj(self._h, os.fsencode(path)), f"load {path}")

    def addMesh(self, pos, nrm, tris) -> int:
        pos = np.ascontiguousarray(pos, np.float32).reshape(-1, 3)
        nrm = np.ascontiguousarray(nrm, np.float32).reshape(-1, 3)
        tris = np.ascontiguousarray(tris, np.int32).reshape(-1, 3)
        return _err(lib().pt_scene_add_mesh(self._h, _fp(pos), _fp(nrm), len(pos), _ip(tris), len(tris)), "addMesh")

    def addModel(self, mesh: int, scale, rot_deg, translate, material, color) -> int:
        mt = MATERIALS[material] if isinstance(material, str) else int(material)
        s = np.array(scale, np.float32); r = np.array(rot_deg, np.float32)
        t = np.array(translate, np.float32); c = np.array(color, np.float32)
        return _err(lib().pt_scene_add_model(self._h, int(mesh), _fp(s), _fp(r), _fp(t), mt, _fp(c)), "addModel")

    def build(self, grid=(25, 25, 25), bvh: bool = True) -> None:
        """addMeshesToGrid (grid) + the per-mesh BLAS that ACCEL_GRID_FAST / ACCEL_BVH
        traverse (``bvh=False``: grid only; allocateOnGPU then adds the BLAS on demand)."""
        g = (ctypes.c_int * 3)(*grid)
        _err(lib().pt_scene_build(self._h, g, 1 if bvh else 0), "build")

    def counts(self) -> dict:
        c = (ctypes.c_int * 9)()
        _err(lib().pt_scene_counts(self._h, c), "counts")
        keys = ["nv", "nt", "nmesh", "nmodel", "ngrid", "nvox", "npv", "nbvh_nodes", "nbvh_refs"]
        return dict(zip(keys, list(c)))

    def export(self) -> dict:
        """Flat copy of Scene.h's member vectors (same layout as oracle.FlatScene)."""
        n = self.counts()
        a = dict(
            vpos=np.zeros((n["nv"], 3), np.float32), vnrm=np.zeros((n["nv"], 3), np.float32),
            tris=np.zeros((n["nt"], 3), np.int32), mesh_ranges=np.zeros((n["nmesh"], 4), np.int32),
            mesh_bbox=np.zeros((n["nmesh"], 6), np.float32), model_ints=np.zeros((n["nmodel"], 3), np.int32),
            model_m2w=np.zeros((n["nmodel"], 16), np.float32), model_w2m=np.zeros((n["nmodel"], 16), np.float32),
            model_color=np.zeros((n["nmodel"], 3), np.float32), grid_ints=np.zeros((n["ngrid"], 4), np.int32),
            grid_vw=np.zeros((n["ngrid"], 3), np.float32), vox=np.zeros((n["nvox"], 3), np.int32),
            per_voxel=np.zeros(max(n["npv"], 1), np.int32))
        _err(lib().pt_scene_export(
            self._h, _fp(a["vpos"]), _fp(a["vnrm"]), _ip(a["tris"]), _ip(a["mesh_ranges"]), _fp(a["mesh_bbox"]),
            _ip(a["model_ints"]), _fp(a["model_m2w"]), _fp(a["model_w2m"]), _fp(a["model_color"]),
            _ip(a["grid_ints"]), _fp(a["grid_vw"]), _ip(a["vox"]), _ip(a["per_voxel"])), "export")
        a["per_voxel"] = a["per_voxel"][:n["npv"]]
        return a


def _scene_export_bvh(self) -> dict:
    n = self.counts()
    nodes = np.zeros((max(n["nbvh_nodes"], 1), 16), np.float32)
    refs = np.zeros(max(n["nbvh_refs"], 1), np.int32)
    roots = np.zeros(max(n["nmesh"], 1), np.int32)
    _err(lib().pt_scene_export_bvh(self._h, _fp(nodes), _ip(refs), _ip(roots)), "export_bvh")
    return dict(nodes=nodes[:n["nbvh_nodes"]], refs=refs[:n["nbvh_refs"]], roots=roots[:n["nmesh"]])


Scene.export_bvh = _scene_export_bvh


def _scene_export_bvh4(self) -> dict:
    """The 4-wide collapse of the BLAS (Bvh4Node: 32 words per node), each
    mesh's 4-wide root (-1: none; the 4-wide traces then refuse the scene) and
    each mesh's first leaf record (`leaf_base`: a leaf link's `first` is
    relative to it)."""
    n = self.counts()
    roots = np.zeros(max(n["nmesh"], 1), np.int32)
    cnt = _err(lib().pt_scene_export_bvh4(self._h, None, _ip(roots)), "export_bvh4")
    nodes = np.zeros((max(cnt, 1), 32), np.float32)
    _err(lib().pt_scene_export_bvh4(self._h, _fp(nodes), _ip(roots)), "export_bvh4")
    base = np.zeros(max(n["nmesh"], 1), np.int32)
    _err(lib().pt_scene_export_bvh4_leaf_base(self._h, _ip(base)), "export_bvh4_leaf_base")
    return dict(nodes=nodes[:cnt], roots=roots[:n["nmesh"]], leaf_base=base[:n["nmesh"]])


Scene.export_bvh4 = _scene_export_bvh4




def selftest_math(x, y) -> np.ndarray:
    """Device evaluation of the kernels' sin/cos/pow/sqrt/div (n x 5)."""
    x = np.ascontiguousarray(x, np.float32); y = np.ascontiguousarray(y, np.float32)
    out = np.zeros((len(x), 5), np.float32)
    _err(lib().pt_selftest_math(len(x), _fp(x), _fp(y), _fp(out)), "selftest_math")
    return out


class Renderer:
    """Renderer (Renderer.h:46-55) on the gfx950 wavefront pipeline."""

    def __init__(self, cfg: RenderConfig | None = None):
        self.cfg = cfg or RenderConfig()
        self._c = self.cfg.c()
        self._h = lib().pt_renderer_create(ctypes.byref(self._c))
        if not self._h:
            _err(-1, "pt_renderer_create")
        self._image_ref = None

    def set_stream(self, hip_stream: int) -> None:
        _err(lib().pt_renderer_set_stream(self._h, ctypes.c_void_p(int(hip_stream))), "set_stream")

    def bind_image(self, device_ptr: int, keepalive=None) -> None:
        self._image_ref = keepalive
        _err(lib().pt_renderer_bind_image(self._h, ctypes.c_void_p(int(device_ptr))), "bind_image")

    def allocateOnGPU(self, scene: Scene) -> None:
        self._scene = scene
        _err(lib().pt_renderer_allocate_on_gpu(self._h, scene._h), "allocateOnGPU")

    def clearImage(self) -> None:
        _err(lib().pt_renderer_clear_image(self._h), "clearImage")

    def renderLoop(self, first_iter: int = 0, n_iters: int | None = None, sync: bool = True) -> None:
        n = self.cfg.iterations if n_iters is None else n_iters
        _err(lib().pt_renderer_render_loop(self._h, int(first_iter), int(n)), "renderLoop")
        if sync:
            self.synchronize()

    def synchronize(self) -> None:
        _err(lib().pt_renderer_synchronize(self._h), "synchronize")

    def image(self) -> np.ndarray:
        out = np.zeros((self.cfg.width * self.cfg.height, 3), np.float32)
        _err(lib().pt_renderer_read_image(self._h, _fp(out)), "read_image")
        return out

    def renderImage(self, path: str = "Render.bmp", iterations_total: int | None = None) -> None:
        it = self.cfg.iterations if iterations_total is None else iterations_total
        _err(lib().pt_renderer_render_image(self._h, os.fsencode(path), int(it)), "renderImage")

    def segments(self) -> int:
        v = lib().pt_renderer_segments(self._h)
        return _err(v, "segments")

    def trace_faults(self) -> int:
        """Persistent-trace waves that gave up at the iteration cap (0 in a correct
        run; non-zero also makes synchronize() / image() raise)."""
        return _err(lib().pt_renderer_trace_faults(self._h), "trace_faults")

    def segments_per_bounce(self, n: int = 64) -> list:
        out = (ctypes.c_longlong * n)()
        _err(lib().pt_renderer_segments_per_bounce(self._h, out, n), "segments_per_bounce")
        return list(out)

    def pipelines(self) -> int:
        """Iterations in flight (own HIP streams) once allocated."""
        return _err(lib().pt_renderer_pipelines(self._h), "pipelines")

    def set_profiling(self, on) -> None:
        """HIP-event timing: False/0 off, True/1 every kernel group, 2 pipeline 0's trace phases only."""
        _err(lib().pt_renderer_set_profiling(self._h, int(on)), "set_profiling")

    def kernel_stats(self) -> dict:
        st = (ctypes.c_double * 11)()
        _err(lib().pt_renderer_kernel_stats_ex(self._h, st, 11), "kernel_stats")
        return dict(bounce_ms=st[0], scan_ms=st[1], primary_ms=st[2],
                    bounce_launches=int(st[3]), scan_launches=int(st[4]),
                    first_ms=st[5], first_launches=int(st[6]),
                    trace_ms=st[7], trace_launches=int(st[8]),
                    sort_ms=st[9], sort_launches=int(st[10]))

    def deferred_rays(self) -> int:
        """Rays k_trace_deferred traced since allocateOnGPU (grid_fast hit sets beyond
        the overflow pool, or undecided walks beyond the hand-on records' room)."""
        return self.segments_per_bounce(_DEFERRED_SLOT + 1)[_DEFERRED_SLOT]

    def primary_hits(self):
        n = self.cfg.width * self.cfg.height
        if self.cfg.tail_drop:
            n = (n // 32) * 32
        d = np.zeros(n, np.float32); nn = np.zeros((n, 3), np.float32); m = np.zeros(n, np.int32)
        _err(lib().pt_renderer_primary_hits(self._h, _fp(d), _fp(nn), _ip(m)), "primary_hits")
        return d, nn, m

    def intersect_rays(self, orig, dirs):
        o = np.ascontiguousarray(orig, np.float32).reshape(-1, 3)
        dd = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
        n = len(o)
        t = np.zeros(n, np.float32); nn = np.zeros((n, 3), np.float32); m = np.zeros(n, np.int32)
        _err(lib().pt_renderer_intersect_rays(self._h, n, _fp(o), _fp(dd), _fp(t), _fp(nn), _ip(m)), "intersect_rays")
        return t, nn, m

    def certify_check(self, orig, dirs):
        """grid_fast test hook: per ray, (fast certificates tried, accepted,
        accepted but disagreeing with the exact walk, full certificates
        disagreeing) -- an (n, 4) int32 array; both disagreement columns must be 0."""
        o = np.ascontiguousarray(orig, np.float32).reshape(-1, 3)
        dd = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
        out = np.zeros((len(o), 4), np.int32)
        _err(lib().pt_renderer_certify_check(self._h, len(o), _fp(o), _fp(dd), _ip(out)), "certify_check")
        return out

    def free(self) -> None:
        if self._h:
            lib().pt_renderer_free(self._h)
            self._h = None

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            try:
                _lib.pt_renderer_free(self._h)
            except Exception:
                pass
            self._h = None


def render(scene_config: str, cfg: RenderConfig | None = None, bmp_out: str | None = "Render.bmp") -> None:
    """main.cpp:11-27 equivalent.  ``cfg=None``: the library's defaults
    (pt_default_config) overlaid with the scene file's RENDER block."""
    c = ctypes.byref(cfg.c()) if cfg is not None else None
    _err(lib().pt_render(os.fsencode(scene_config), c, os.fsencode(bmp_out) if bmp_out else None), "render")
