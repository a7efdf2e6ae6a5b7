"""CPU oracle for the PathTracerAP bounce loop -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker: the product
(``pathtracerap_amd``) never imports, links or calls it.

What lives here:

* ``libptoracle.so`` (built from ``ptoracle.c`` by ``make -C oracle``): a
  plain-C restatement of the reference's render loop (Renderer.cpp /
  utility.h / glm / thrust semantics), see ``ptoracle.h``.
* ``load_obj``: restatement of Scene::loadAndProcessMeshFile + processMesh
  (Scene.cpp:226-291) with Assimp's OBJ importer semantics (one vertex per
  face corner, positions and normals scaled by BASE_MODEL_SCALE).
* ``reference_scene``: the hard-coded scene of Scene::Scene (Scene.cpp:3-224).
* ``build_scene``: model matrices (glm restatement) + addMeshesToGrid.

Pinning: the reference is unbuildable here (CUDA toolkit, thrust, Assimp), so
the oracle is pinned against the reference's own output image
``PathTracerAP/Render.bmp`` (1000x800, ITER=500, Scene.cpp scene), committed
as ``tests/golden/reference_render_1000x800_500.npz`` -- see
``tests/test_oracle_golden.py`` and ``tests/golden/make_golden.py``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libptoracle.so")

# Primitive.h:70-79
MATERIALS = {
    "DIFFUSE": 0, "SPECULAR": 1, "REFLECTIVE": 2, "REFRACTIVE": 3,
    "EMISSIVE": 4, "COAT": 5, "METAL": 6,
}
BASE_MODEL_SCALE = np.float32(1000.0)   # Config.h:16
GRID_DIM = (25, 25, 25)                  # Config.h:8-10


def build(force: bool = False) -> str:
    """Compile libptoracle.so in place (gcc)."""
    if force or not os.path.exists(_LIB_PATH) or (
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "ptoracle.c"))):
        subprocess.check_call(["make", "-s", "-C", _HERE], stdout=subprocess.DEVNULL)
    return _LIB_PATH


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.ptor_sinf.restype = ctypes.c_float
        _lib.ptor_sinf.argtypes = [ctypes.c_float]
        _lib.ptor_cosf.restype = ctypes.c_float
        _lib.ptor_cosf.argtypes = [ctypes.c_float]
        _lib.ptor_powf.restype = ctypes.c_float
        _lib.ptor_powf.argtypes = [ctypes.c_float, ctypes.c_float]
        _lib.ptor_hash.restype = ctypes.c_uint
        _lib.ptor_hash.argtypes = [ctypes.c_uint]
        _lib.ptor_u01_first.restype = ctypes.c_float
        _lib.ptor_u01_first.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    return _lib


_P_F = ctypes.POINTER(ctypes.c_float)
_P_I = ctypes.POINTER(ctypes.c_int)


class _CScene(ctypes.Structure):
    _fields_ = [
        ("nv", ctypes.c_int), ("vpos", _P_F), ("vnrm", _P_F),
        ("nt", ctypes.c_int), ("tris", _P_I),
        ("nmesh", ctypes.c_int), ("mesh_ranges", _P_I), ("mesh_bbox", _P_F),
        ("nmodel", ctypes.c_int), ("model_ints", _P_I), ("model_m2w", _P_F),
        ("model_w2m", _P_F), ("model_color", _P_F),
        ("ngrid", ctypes.c_int), ("grid_ints", _P_I), ("grid_vw", _P_F),
        ("nvox", ctypes.c_int), ("vox", _P_I),
        ("npv", ctypes.c_int), ("per_voxel", _P_I),
        ("gdim", ctypes.c_int * 3),
    ]


class _CConfig(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int), ("height", ctypes.c_int),
        ("first_iter", ctypes.c_int), ("iterations", ctypes.c_int),
        ("max_bounces", ctypes.c_int), ("accel", ctypes.c_int),
        ("threads", ctypes.c_int), ("tail_drop", ctypes.c_int),
        ("cam", ctypes.c_double * 3), ("plane_z", ctypes.c_double),
        ("plane_x0", ctypes.c_double), ("plane_y0", ctypes.c_double),
        ("plane_w", ctypes.c_double), ("plane_h", ctypes.c_double),
    ]


def _fp(a):
    return a.ctypes.data_as(_P_F)


def _ip(a):
    return a.ctypes.data_as(_P_I)


# --------------------------------------------------------------------------
# Scene description
# --------------------------------------------------------------------------

@dataclass
class FlatScene:
    """Scene.h member vectors, flattened (same layout as the C-ABI export)."""
    vpos: np.ndarray            # (nv,3) f32
    vnrm: np.ndarray            # (nv,3) f32
    tris: np.ndarray            # (nt,3) i32
    mesh_ranges: np.ndarray     # (nmesh,4) i32  vs ve ts te
    mesh_bbox: np.ndarray       # (nmesh,6) f32  min3 max3
    model_ints: np.ndarray      # (nmodel,3) i32 mesh grid mattype
    model_m2w: np.ndarray       # (nmodel,16) f32 column-major
    model_w2m: np.ndarray       # (nmodel,16) f32
    model_color: np.ndarray     # (nmodel,3) f32
    grid_ints: np.ndarray       # (ngrid,4) i32 vox_s vox_e etype eidx
    grid_vw: np.ndarray         # (ngrid,3) f32
    vox: np.ndarray             # (nvox,3) i32 start end etype
    per_voxel: np.ndarray       # (npv,) i32
    gdim: tuple = GRID_DIM
    _keep: list = field(default_factory=list, repr=False)

    def c(self) -> _CScene:
        arrs = {}
        for k in ("vpos", "vnrm", "mesh_bbox", "model_m2w", "model_w2m", "model_color", "grid_vw"):
            arrs[k] = np.ascontiguousarray(getattr(self, k), dtype=np.float32)
        for k in ("tris", "mesh_ranges", "model_ints", "grid_ints", "vox", "per_voxel"):
            arrs[k] = np.ascontiguousarray(getattr(self, k), dtype=np.int32)
            if arrs[k].size == 0:
                arrs[k] = np.zeros(1, np.int32)
        self._keep = list(arrs.values())
        s = _CScene()
        s.nv = len(self.vpos); s.vpos = _fp(arrs["vpos"]); s.vnrm = _fp(arrs["vnrm"])
        s.nt = len(self.tris); s.tris = _ip(arrs["tris"])
        s.nmesh = len(self.mesh_ranges); s.mesh_ranges = _ip(arrs["mesh_ranges"]); s.mesh_bbox = _fp(arrs["mesh_bbox"])
        s.nmodel = len(self.model_ints); s.model_ints = _ip(arrs["model_ints"])
        s.model_m2w = _fp(arrs["model_m2w"]); s.model_w2m = _fp(arrs["model_w2m"])
        s.model_color = _fp(arrs["model_color"])
        s.ngrid = len(self.grid_ints); s.grid_ints = _ip(arrs["grid_ints"]); s.grid_vw = _fp(arrs["grid_vw"])
        s.nvox = len(self.vox); s.vox = _ip(arrs["vox"])
        s.npv = len(self.per_voxel); s.per_voxel = _ip(arrs["per_voxel"])
        s.gdim[0], s.gdim[1], s.gdim[2] = self.gdim
        return s


@dataclass
class RenderConfig:
    width: int = 1000               # Config.h:12
    height: int = 800               # Config.h:13
    iterations: int = 500           # Config.h:19 ITER
    first_iter: int = 0
    max_bounces: int = 5            # Renderer.cpp:550
    accel: int = 0                  # 0 grid (reference), 1 exact closest hit
    threads: int = 0
    tail_drop: int = 0
    cam: tuple = (0.0, 0.0, 920.0)  # Renderer.cpp:528
    plane_z: float = 900.0          # Renderer.cpp:543
    plane_x0: float = -10.0         # Renderer.cpp:541
    plane_y0: float = -4.0          # Renderer.cpp:542
    plane_w: float = 20.0           # Renderer.cpp:538
    plane_h: float = 16.0           # Renderer.cpp:539

    def c(self) -> _CConfig:
        c = _CConfig()
        c.width, c.height = self.width, self.height
        c.first_iter, c.iterations = self.first_iter, self.iterations
        c.max_bounces, c.accel, c.threads, c.tail_drop = self.max_bounces, self.accel, self.threads, self.tail_drop
        c.cam[0], c.cam[1], c.cam[2] = self.cam
        c.plane_z, c.plane_x0, c.plane_y0, c.plane_w, c.plane_h = (
            self.plane_z, self.plane_x0, self.plane_y0, self.plane_w, self.plane_h)
        return c


def load_obj(path: str):
    """Scene::loadAndProcessMeshFile + processMesh (Scene.cpp:226-291) with
    Assimp OBJ importer semantics: every face corner becomes its own vertex
    (no aiProcess_JoinIdenticalVertices), position/normal scaled by
    BASE_MODEL_SCALE.  Decimal text -> double -> float.  Polygons are fan-
    triangulated and corners without ``vn`` get the face's geometric normal
    (both are extensions: the reference asserts triangles with normals).
    Returns (pos (n,3) f32, nrm (n,3) f32, tris (m,3) i32 local indices)."""
    vs, vns = [], []
    faces = []
    with open(path, "r") as f:
        for line in f:
            if line.startswith("v "):
                p = line.split()
                vs.append((float(p[1]), float(p[2]), float(p[3])))
            elif line.startswith("vn "):
                p = line.split()
                vns.append((float(p[1]), float(p[2]), float(p[3])))
            elif line.startswith("f "):
                corners = []
                for tok in line.split()[1:]:
                    parts = tok.split("/")
                    vi = int(parts[0])
                    vi = vi - 1 if vi > 0 else len(vs) + vi
                    ni = -1
                    if len(parts) >= 3 and parts[2] != "":
                        ni = int(parts[2])
                        ni = ni - 1 if ni > 0 else len(vns) + ni
                    corners.append((vi, ni))
                faces.append(corners)
    V = np.array(vs, dtype=np.float64).astype(np.float32).reshape(-1, 3)
    N = np.array(vns, dtype=np.float64).astype(np.float32).reshape(-1, 3)
    pos, nrm, tris = [], [], []
    base = 0
    for corners in faces:
        k = len(corners)
        cp = [V[c[0]] for c in corners]
        need_geo = any(c[1] < 0 for c in corners)
        if need_geo:
            g = _geo_normal(cp[0], cp[1], cp[2])
        for j, c in enumerate(corners):
            pos.append(cp[j])
            nrm.append(N[c[1]] if c[1] >= 0 else g)
        for j in range(1, k - 1):
            tris.append((base, base + j, base + j + 1))
        base += k
    pos = np.array(pos, dtype=np.float32).reshape(-1, 3) * BASE_MODEL_SCALE
    nrm = np.array(nrm, dtype=np.float32).reshape(-1, 3) * BASE_MODEL_SCALE
    return pos.astype(np.float32), nrm.astype(np.float32), np.array(tris, dtype=np.int32).reshape(-1, 3)


def _geo_normal(p0, p1, p2):
    f = np.float32
    e1 = (p1 - p0).astype(np.float32)
    e2 = (p2 - p0).astype(np.float32)
    c = np.array([f(e1[1] * e2[2]) - f(e2[1] * e1[2]),
                  f(e1[2] * e2[0]) - f(e2[2] * e1[0]),
                  f(e1[0] * e2[1]) - f(e2[0] * e1[1])], dtype=np.float32)
    d = f(f(f(c[0] * c[0]) + f(c[1] * c[1])) + f(c[2] * c[2]))
    s = f(f(1.0) / np.sqrt(d, dtype=np.float32))
    return (c * s).astype(np.float32)


def _bbox_sequential(pos):
    """BoundingBox() + update() over the vertices in order (Primitive.h:35-60):
    min = min > v ? v : min starting at FLOAT_MAX (max symmetric at FLOAT_MIN).
    The survivor is the FIRST vertex holding the extreme value (keeps its sign
    of zero); NaN never replaces."""
    mn = np.full(3, 9999999.0, np.float32)
    mx = np.full(3, -9999990.0, np.float32)
    for a in range(3):
        col = pos[:, a] if len(pos) else np.zeros(0, np.float32)
        ok = ~np.isnan(col)
        if ok.any():
            m = col[ok].min()
            if m < mn[a]:
                mn[a] = col[np.nonzero(col == m)[0][0]]
            M = col[ok].max()
            if M > mx[a]:
                mx[a] = col[np.nonzero(col == M)[0][0]]
    return mn, mx


def model_matrix(scale, rot_deg, translate):
    """glm translate*rotate*scale and inverse (Scene.cpp:34-39), in C."""
    m2w = np.zeros(16, np.float32)
    w2m = np.zeros(16, np.float32)
    s = np.array(scale, np.float32); r = np.array(rot_deg, np.float32); t = np.array(translate, np.float32)
    lib().ptor_model_matrix(_fp(s), _fp(r), _fp(t), _fp(m2w), _fp(w2m))
    return m2w, w2m


def build_scene(meshes, models, gdim=GRID_DIM) -> FlatScene:
    """meshes: list of (pos, nrm, tris_local); models: list of dicts with
    mesh, scale, rot, translate, material (name), color.  Mirrors
    Scene::Scene's vectors (Scene.cpp:6-223) and addMeshesToGrid."""
    vpos, vnrm, tris, ranges, bbox = [], [], [], [], []
    nv = 0
    nt = 0
    for pos, nrm, tl in meshes:
        vs_, ve = nv, nv + len(pos)
        ts, te = nt, nt + len(tl)
        vpos.append(pos); vnrm.append(nrm); tris.append(tl + nv)
        mn, mx = _bbox_sequential(pos)
        ranges.append((vs_, ve, ts, te)); bbox.append(np.concatenate([mn, mx]))
        nv, nt = ve, te
    vpos = np.concatenate(vpos).astype(np.float32) if vpos else np.zeros((0, 3), np.float32)
    vnrm = np.concatenate(vnrm).astype(np.float32) if vnrm else np.zeros((0, 3), np.float32)
    tris = np.concatenate(tris).astype(np.int32) if tris else np.zeros((0, 3), np.int32)
    ranges = np.array(ranges, np.int32).reshape(-1, 4)
    bbox = np.array(bbox, np.float32).reshape(-1, 6)
    nmodel = len(models)
    model_ints = np.zeros((nmodel, 3), np.int32)
    m2w = np.zeros((nmodel, 16), np.float32); w2m = np.zeros((nmodel, 16), np.float32)
    color = np.zeros((nmodel, 3), np.float32)
    for i, m in enumerate(models):
        model_ints[i, 0] = m["mesh"]
        model_ints[i, 2] = MATERIALS[m["material"]]
        a, b = model_matrix(m["scale"], m.get("rot", (0, 0, 0)), m["translate"])
        m2w[i] = a; w2m[i] = b
        color[i] = np.array(m["color"], np.float32)
    G = int(np.prod(gdim))
    nmesh = len(ranges)
    grid_ints = np.zeros((max(nmesh, 1), 4), np.int32)
    grid_vw = np.zeros((max(nmesh, 1), 3), np.float32)
    vox = np.zeros((max(nmesh, 1) * G, 3), np.int32)
    cap = 1 << 20
    gd = (ctypes.c_int * 3)(*gdim)
    while True:
        pv = np.zeros(cap, np.int32)
        ng, nvx, npv = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        rc = lib().ptor_build_grids(
            nmesh, _ip(ranges), _fp(bbox), _fp(vpos), _ip(tris), nmodel, _ip(model_ints), gd,
            ctypes.byref(ng), _ip(grid_ints), _fp(grid_vw), ctypes.byref(nvx), _ip(vox),
            cap, ctypes.byref(npv), _ip(pv))
        if rc >= 0:
            break
        cap = -rc
    return FlatScene(vpos=vpos, vnrm=vnrm, tris=tris, mesh_ranges=ranges, mesh_bbox=bbox,
                     model_ints=model_ints, model_m2w=m2w, model_w2m=w2m, model_color=color,
                     grid_ints=grid_ints[:ng.value].copy(), grid_vw=grid_vw[:ng.value].copy(),
                     vox=vox[:nvx.value].copy(), per_voxel=pv[:npv.value].copy(), gdim=tuple(gdim))


# Scene::Scene (Scene.cpp:6-221): meshes box(0), ceiling_light(1), monkey(2);
# models in push_back order.
REFERENCE_MESH_FILES = ["enclosing_box.obj", "ceiling_light.obj", "blender_monkey.obj"]
REFERENCE_MODELS = [
    dict(mesh=2, scale=(0.08, 0.08, 0.08), rot=(0, 45, 0), translate=(-50, -25, 150), material="METAL", color=(0.001, 0.99, 0.2)),
    dict(mesh=2, scale=(0.1, 0.1, 0.1), rot=(0, -40, 0), translate=(75, 100, 0), material="COAT", color=(0.99, 0.99, 0.001)),
    dict(mesh=2, scale=(0.1, 0.1, 0.1), rot=(0, 0, 0), translate=(325, 45, 0), material="REFLECTIVE", color=(0.99, 0.99, 0.75)),
    dict(mesh=0, scale=(0.1, 0.1, 0.1), rot=(0, 180, 0), translate=(25, -120, 0), material="DIFFUSE", color=(0.99, 0.99, 0.99)),
    dict(mesh=1, scale=(0.1, 0.1, 0.1), rot=(0, 45, 0), translate=(325, -120, 0), material="DIFFUSE", color=(0.99, 0.50, 0.60)),
    dict(mesh=1, scale=(0.1, 0.1, 0.1), rot=(0, 45, 0), translate=(-225, 8, 0), material="COAT", color=(0.40, 0.10, 0.99)),
    dict(mesh=1, scale=(0.1, 0.1, 0.1), rot=(0, 30, 0), translate=(75, -90, 0), material="METAL", color=(0.99, 0.05, 0.10)),
    dict(mesh=1, scale=(0.2, 0.1, 0.2), rot=(0, 0, 0), translate=(0, 850, -100), material="EMISSIVE", color=(0.99, 0.99, 0.99)),
    dict(mesh=1, scale=(0.2, 0.2, 0.1), rot=(0, 0, 0), translate=(0, 375, 950), material="EMISSIVE", color=(0.99, 0.99, 0.99)),
    dict(mesh=1, scale=(0.1, 0.2, 0.2), rot=(0, 0, 0), translate=(-520, 375, 0), material="EMISSIVE", color=(0.99, 0.99, 0.99)),
    dict(mesh=1, scale=(0.1, 0.2, 0.2), rot=(0, 0, 0), translate=(550, 375, 0), material="EMISSIVE", color=(0.99, 0.99, 0.99)),
]


def reference_scene(input_dir: str, gdim=GRID_DIM) -> FlatScene:
    meshes = [load_obj(os.path.join(input_dir, f)) for f in REFERENCE_MESH_FILES]
    return build_scene(meshes, REFERENCE_MODELS, gdim)


# --------------------------------------------------------------------------
# Rendering / intersection entry points
# --------------------------------------------------------------------------

def render(scene: FlatScene, cfg: RenderConfig, image: np.ndarray | None = None):
    """renderLoop: returns (accumulated image (H*W,3) f32, ray segments)."""
    if image is None:
        image = np.zeros((cfg.width * cfg.height, 3), np.float32)
    cs = scene.c()
    cc = cfg.c()
    seg = ctypes.c_longlong(0)
    rc = lib().ptor_render(ctypes.byref(cs), ctypes.byref(cc), _fp(image), ctypes.byref(seg))
    if rc != 0:
        raise RuntimeError("ptor_render failed")
    return image, seg.value


def intersect_primary(scene: FlatScene, cfg: RenderConfig):
    n = cfg.width * cfg.height
    dist = np.zeros(n, np.float32); nrm = np.zeros((n, 3), np.float32); model = np.zeros(n, np.int32)
    cs = scene.c(); cc = cfg.c()
    lib().ptor_intersect_primary(ctypes.byref(cs), ctypes.byref(cc), _fp(dist), _fp(nrm), _ip(model))
    return dist, nrm, model


def intersect_rays(scene: FlatScene, orig, dirs, accel=0, threads=0):
    orig = np.ascontiguousarray(orig, np.float32); dirs = np.ascontiguousarray(dirs, np.float32)
    n = len(orig)
    dist = np.zeros(n, np.float32); nrm = np.zeros((n, 3), np.float32); model = np.zeros(n, np.int32)
    cs = scene.c()
    lib().ptor_intersect_rays(ctypes.byref(cs), accel, n, _fp(orig), _fp(dirs), _fp(dist), _fp(nrm), _ip(model), threads)
    return dist, nrm, model


def to_bmp_bytes(image: np.ndarray, width: int, height: int, iterations: int) -> bytes:
    """Renderer::renderImage (Renderer.cpp:15-63): 54-byte header, rows
    bottom-up, bytes (x,y,z) of (sum * (1/ITER)) * 255 truncated to char."""
    div = np.float32(1.0) / np.float32(iterations)
    c = (image.astype(np.float32) * div).astype(np.float32) * np.float32(255.0)
    ci = np.where(np.isfinite(c) & (c < 2147483648.0) & (c >= -2147483648.0), c, -2147483648.0)
    b = (np.trunc(ci).astype(np.int64) & 0xFF).astype(np.uint8)
    hdr = bytearray(54)
    hdr[0:2] = b"BM"
    hdr[10] = 54
    hdr[14] = 40
    hdr[18:22] = int(width).to_bytes(4, "little", signed=True)
    hdr[22:26] = int(height).to_bytes(4, "little", signed=True)
    hdr[26] = 1
    hdr[28] = 24
    hdr[2:6] = (54 + 3 * width * height).to_bytes(4, "little", signed=True)
    hdr[34:38] = (3 * width * height).to_bytes(4, "little", signed=True)
    return bytes(hdr) + b.reshape(-1).tobytes()
