"""Synthetic OBJ scenes for the BASELINE.json configurations.

No datasets can be downloaded, so the benchmark meshes are procedural:
a displaced torus of ``2 * nu * nv`` triangles (smooth per-vertex normals)
inside an open-front room with emissive ceiling panels, laid out like the
reference's Scene.cpp room (enclosing box scaled 0.1 at y = -120, lights
above).  Meshes are written as Wavefront OBJ (``v`` / ``vn`` / ``f a//a``)
and loaded through the same loader as user files (Scene::loadObj =
Scene.cpp:226-291 semantics).
"""
from __future__ import annotations

import os

import numpy as np


def torus_mesh(ntri: int, major: float = 2.5, minor: float = 0.9, bumps: float = 0.08, seed: int = 0):
    """Displaced torus with about ``ntri`` triangles (OBJ units, pre x1000)."""
    nv = max(3, int(round(np.sqrt(ntri / 4.0))))
    nu = max(3, int(round(ntri / (2.0 * nv))))
    u = np.linspace(0, 2 * np.pi, nu, endpoint=False)
    v = np.linspace(0, 2 * np.pi, nv, endpoint=False)
    U, V = np.meshgrid(u, v, indexing="ij")
    rng = np.random.RandomState(seed)
    ph = rng.uniform(0, 2 * np.pi, 4)
    r = minor * (1.0 + bumps * (np.sin(7 * U + ph[0]) * np.cos(5 * V + ph[1])
                               + 0.5 * np.sin(23 * U + ph[2]) * np.sin(17 * V + ph[3])))
    x = (major + r * np.cos(V)) * np.cos(U)
    y = r * np.sin(V)
    z = (major + r * np.cos(V)) * np.sin(U)
    P = np.stack([x, y, z], -1)
    # smooth normals from finite differences on the periodic grid
    du = np.roll(P, -1, 0) - np.roll(P, 1, 0)
    dv = np.roll(P, -1, 1) - np.roll(P, 1, 1)
    N = np.cross(dv, du)
    N /= np.linalg.norm(N, axis=-1, keepdims=True)
    idx = np.arange(nu * nv).reshape(nu, nv)
    a = idx
    b = np.roll(idx, -1, 0)
    c = np.roll(np.roll(idx, -1, 0), -1, 1)
    d = np.roll(idx, -1, 1)
    tris = np.concatenate([np.stack([a, b, c], -1).reshape(-1, 3), np.stack([a, c, d], -1).reshape(-1, 3)])
    return P.reshape(-1, 3).astype(np.float32), N.reshape(-1, 3).astype(np.float32), tris.astype(np.int32)


def room_mesh():
    """Open-front room (floor, ceiling, back, left, right slabs), x,z in [-5,5], y in [0,10]."""
    slabs = [((-5.25, -0.25, -5.25), (5.25, 0.0, 5.25)),     # floor
             ((-5.25, 10.0, -5.25), (5.25, 10.25, 5.25)),    # ceiling
             ((-5.25, 0.0, -5.25), (5.25, 10.0, -5.0)),      # back
             ((-5.25, 0.0, -5.0), (-5.0, 10.0, 5.25)),       # left
             ((5.0, 0.0, -5.0), (5.25, 10.0, 5.25))]         # right
    return _boxes(slabs)


def light_mesh():
    return _boxes([((-1.0, -1.0, -1.0), (1.0, 1.0, 1.0))])


def _boxes(boxes):
    P, N, T = [], [], []
    for lo, hi in boxes:
        for axis in range(3):
            for side in (0, 1):
                u, w = (axis + 1) % 3, (axis + 2) % 3
                n = [0.0, 0.0, 0.0]
                n[axis] = 1.0 if side else -1.0
                quad = []
                for qu, qw in ((0, 0), (1, 0), (1, 1), (0, 1)):
                    p = [0.0, 0.0, 0.0]
                    p[axis] = hi[axis] if side else lo[axis]
                    p[u] = hi[u] if qu else lo[u]
                    p[w] = hi[w] if qw else lo[w]
                    quad.append(p)
                base = len(P)
                P.extend(quad)
                N.extend([n] * 4)
                if side:
                    T.extend([(base, base + 1, base + 2), (base, base + 2, base + 3)])
                else:
                    T.extend([(base, base + 2, base + 1), (base, base + 3, base + 2)])
    return np.array(P, np.float32), np.array(N, np.float32), np.array(T, np.int32)


def write_obj(path: str, pos, nrm, tris) -> None:
    with open(path, "w") as f:
        f.write("# synthetic mesh (pathtracerap_amd.synthetic)\n")
        np.savetxt(f, pos, fmt="v %.6f %.6f %.6f")
        np.savetxt(f, nrm, fmt="vn %.6f %.6f %.6f")
        t = tris + 1
        np.savetxt(f, np.stack([t[:, 0], t[:, 0], t[:, 1], t[:, 1], t[:, 2], t[:, 2]], 1),
                   fmt="f %d//%d %d//%d %d//%d")


def _write_atomic(path, pos, nrm, tris):
    tmp = f"{path}.{os.getpid()}.tmp"
    write_obj(tmp, pos, nrm, tris)
    os.replace(tmp, path)


def diffuse_scene(out_dir: str, ntri: int = 100_000, seed: int = 0, width: int = 1280, height: int = 1024,
                  iterations: int = 256, bounces: int = 8, accel: str = "grid_fast", metallic: bool = False) -> str:
    """Writes the OBJs and a Config.txt-grammar scene file; returns its path.

    configs[1]: diffuse-only OBJ (~100k tris), 1280x1024, 256 spp, 8 bounces.
    ``metallic=True`` adds METAL/COAT/REFLECTIVE instances (configs[2]-style).
    """
    os.makedirs(out_dir, exist_ok=True)
    tag = f"torus_{ntri}_{seed}"
    obj = os.path.join(out_dir, tag + ".obj")
    if not os.path.exists(obj):
        _write_atomic(obj, *torus_mesh(ntri, seed=seed))
    for name, fn in (("room", room_mesh), ("light", light_mesh)):
        p = os.path.join(out_dir, name + ".obj")
        if not os.path.exists(p):
            _write_atomic(p, *fn())
    lines = [
        "# synthetic scene (pathtracerap_amd.synthetic.diffuse_scene)",
        "", "RENDER", f"resolution:[{width},{height}]", f"iterations:{iterations}",
        f"bounces:{bounces}", "grid:[25,25,25]", f"accel:{accel}",
        "", "OBJ", "room", "room.obj", "", "OBJ", "light", "light.obj", "", "OBJ", "torus", tag + ".obj",
        "", "DIFFUSE", "wall", "[0.85, 0.85, 0.85]",
        "", "DIFFUSE", "red", "[0.85, 0.15, 0.12]",
        "", "DIFFUSE", "torus_mat", "[0.75, 0.62, 0.40]",
        "", "EMISSIVE", "lamp", "[0.99, 0.99, 0.99]",
        "", "METAL", "chrome", "[0.90, 0.90, 0.95]",
        "", "COAT", "blue_coat", "[0.15, 0.30, 0.90]",
        "", "MESH", "room_model", "room", "translate:[0,-120,0]", "scale:[0.1,0.1,0.1]", "material:wall",
        "", "MESH", "torus_model", "torus", "translate:[0,130,0]", "rotate:[35,20,0]", "scale:[0.1,0.1,0.1]",
        "material:" + ("chrome" if metallic else "torus_mat"),
        "", "MESH", "lamp_model", "light", "translate:[0,870,-50]", "scale:[0.2,0.02,0.2]", "material:lamp",
        "", "MESH", "lamp_front", "light", "translate:[0,375,950]", "scale:[0.2,0.2,0.1]", "material:lamp",
        "", "MESH", "block", "light", "translate:[-300,-60,150]", "rotate:[0,30,0]", "scale:[0.06,0.06,0.06]",
        "material:" + ("blue_coat" if metallic else "red"),
    ]
    path = os.path.join(out_dir, f"scene_{tag}{'_metal' if metallic else ''}.txt")
    tmp = f"{path}.{os.getpid()}.tmp"          # atomic: another process may be reading the old file
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, path)
    return path


# Models of diffuse_scene, in the order its MESH blocks add them:
# (mesh, translate, rotate, scale, material, color); metallic swaps in the second pair.
_MODELS = [
    ("room", (0, -120, 0), (0, 0, 0), (0.1, 0.1, 0.1), ("DIFFUSE", (0.85, 0.85, 0.85)), None),
    ("torus", (0, 130, 0), (35, 20, 0), (0.1, 0.1, 0.1), ("DIFFUSE", (0.75, 0.62, 0.40)), ("METAL", (0.90, 0.90, 0.95))),
    ("light", (0, 870, -50), (0, 0, 0), (0.2, 0.02, 0.2), ("EMISSIVE", (0.99, 0.99, 0.99)), None),
    ("light", (0, 375, 950), (0, 0, 0), (0.2, 0.2, 0.1), ("EMISSIVE", (0.99, 0.99, 0.99)), None),
    ("light", (-300, -60, 150), (0, 30, 0), (0.06, 0.06, 0.06), ("DIFFUSE", (0.85, 0.15, 0.12)), ("COAT", (0.15, 0.30, 0.90))),
]


def build_scene(P, ntri: int = 100_000, seed: int = 0, metallic: bool = False, grid=(25, 25, 25), bvh: bool = True):
    """diffuse_scene's layout built in memory (Scene.addMesh / addModel, no OBJ
    round trip): for the 10M-triangle configs[4] scene, whose OBJ text would take
    about a minute to write and parse.  Same meshes, transforms and materials; the
    vertex coordinates are the float32 values themselves rather than their 6-digit
    OBJ text, so the geometry differs from diffuse_scene's by that rounding."""
    s = P.Scene()
    meshes = {"room": s.addMesh(*room_mesh()), "light": s.addMesh(*light_mesh()),
              "torus": s.addMesh(*torus_mesh(ntri, seed=seed))}
    for mesh, tr, rot, sc, mat, alt in _MODELS:
        name, color = alt if (metallic and alt) else mat
        s.addModel(meshes[mesh], sc, rot, tr, name, color)
    s.build(grid=grid, bvh=bvh)
    return s
