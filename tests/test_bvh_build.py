"""BLAS structure checks (host builder, CPU): every triangle referenced once,
every triangle's tolerance-grown bounds inside its leaf box, depth within the
kernels' LDS stack."""
import numpy as np
import pytest

from conftest import REF_SCENE


def _walk(nodes, root):
    ints = nodes.view(np.int32)
    leaves, depth_max = [], 0
    stack = [(root, 1)]
    while stack:
        n, d = stack.pop()
        depth_max = max(depth_max, d)
        for c, (lo, hi, link, cnt) in enumerate([(slice(0, 3), slice(4, 7), 3, 11), (slice(8, 11), slice(12, 15), 7, 15)]):
            count = ints[n, cnt]
            if count < 0:
                continue
            box = (nodes[n, lo], nodes[n, hi])
            if count == 0:
                stack.append((ints[n, link], d + 1))
            else:
                leaves.append((ints[n, link], count, box))
    return leaves, depth_max


@pytest.mark.parametrize("ntri", [10, 5000, 60000])
def test_bvh_covers_every_triangle(pt_mod, ntri):
    from pathtracerap_amd.synthetic import torus_mesh
    pos, nrm, tris = torus_mesh(ntri, seed=1)
    s = pt_mod.Scene()
    m = s.addMesh(pos, nrm, tris)
    s.addModel(m, (1, 1, 1), (0, 0, 0), (0, 0, 0), "DIFFUSE", (1, 1, 1))
    s.build(bvh=True)
    b = s.export_bvh()
    a = s.export()
    leaves, depth = _walk(b["nodes"], b["roots"][0])
    assert depth <= 23          # kernels' LDS stack holds 24 entries
    seen = np.zeros(len(a["tris"]), np.int32)
    V = a["vpos"].astype(np.float64)
    for first, cnt, (lo, hi) in leaves:
        for t in b["refs"][first:first + cnt]:
            seen[t] += 1
            p = V[a["tris"][t]]
            e1, e2 = p[1] - p[0], p[2] - p[0]
            for u, v in ((-0.005, -0.005), (1.01, -0.005), (-0.005, 1.01)):
                q = p[0] + u * e1 + v * e2
                assert (q >= lo - 1e-9).all() and (q <= hi + 1e-9).all()
    assert (seen == 1).all()


def test_reference_scene_bvh(pt_mod):
    s = pt_mod.Scene(REF_SCENE)
    s.build(bvh=True)
    b = s.export_bvh()
    c = s.counts()
    # every triangle once; 64-byte leaf records (PT_TRI_REC 4) add padding slots (triangle -1)
    assert (b["refs"] >= 0).sum() == c["nt"] and c["nbvh_refs"] >= c["nt"]
    for r in b["roots"]:
        _, depth = _walk(b["nodes"], r)
        assert depth <= 23


def test_depth_cap_on_degenerate_distribution(pt_mod):
    """Pathological input (all triangles stacked on one line of centroids)
    still respects the depth cap."""
    n = 4000
    z = np.repeat(np.arange(n // 2, dtype=np.float32), 2) * 1e-3
    pos = np.zeros((3 * n, 3), np.float32)
    pos[0::3] = np.c_[np.zeros(n), np.zeros(n), z]
    pos[1::3] = np.c_[np.ones(n), np.zeros(n), z]
    pos[2::3] = np.c_[np.zeros(n), np.ones(n), z]
    nrm = np.tile(np.float32([0, 0, 1]), (3 * n, 1))
    tris = np.arange(3 * n, dtype=np.int32).reshape(-1, 3)
    s = pt_mod.Scene()
    m = s.addMesh(pos, nrm, tris)
    s.addModel(m, (1, 1, 1), (0, 0, 0), (0, 0, 0), "DIFFUSE", (1, 1, 1))
    s.build(bvh=True)
    b = s.export_bvh()
    leaves, depth = _walk(b["nodes"], b["roots"][0])
    assert depth <= 23
    assert sum(c for _, c, _ in leaves) == n




def _walk4(nodes, root, base=0):
    """Leaves (first, count, box) and depth of a 4-wide BLAS (Bvh4Node rows);
    `base` = the mesh's leaf_base, which the mesh-relative leaf links add back."""
    ints = nodes.view(np.int32)
    leaves, depth_max, seen = [], 0, set()
    stack = [(root, 1)]
    while stack:
        n, d = stack.pop()
        assert n not in seen            # a tree: every node reached once
        seen.add(n)
        depth_max = max(depth_max, d)
        for c in range(4):
            count = ints[n, 28 + c]
            if count < 0:
                continue
            box = (nodes[n, [c, 4 + c, 8 + c]], nodes[n, [12 + c, 16 + c, 20 + c]])
            if count == 0:
                stack.append((ints[n, 24 + c], d + 1))
            else:                          # a leaf's link is its stack entry: 1 << 31 | count << 26 | first
                e = int(ints[n, 24 + c]) & 0xFFFFFFFF
                assert e >> 31 == 1 and (e >> 26) & 31 == count
                leaves.append((base + (e & ((1 << 26) - 1)), count, box))
    return leaves, depth_max, seen


@pytest.mark.parametrize("order", ["0", "1"])
@pytest.mark.parametrize("ntri", [10, 5000, 60000])
def test_bvh4_collapse_keeps_every_leaf_box_bit_for_bit(pt_mod, monkeypatch, ntri, order):
    """The 4-wide BLAS (k_trace_gf's node steps) holds exactly the binary
    BLAS's leaves, with the same boxes bit for bit, in fewer nodes; every
    leaf fits the traversal stack's leaf encoding.  Breadth-first (default)
    and depth-first (PT_BVH4_ORDER=1) node numbering alike."""
    monkeypatch.setenv("PT_BVH4_ORDER", order)
    from pathtracerap_amd.synthetic import torus_mesh
    pos, nrm, tris = torus_mesh(ntri, seed=1)
    s = pt_mod.Scene()
    m = s.addMesh(pos, nrm, tris)
    s.addModel(m, (1, 1, 1), (0, 0, 0), (0, 0, 0), "DIFFUSE", (1, 1, 1))
    s.build(bvh=True)
    b, b4 = s.export_bvh(), s.export_bvh4()
    leaves2, depth2 = _walk(b["nodes"], b["roots"][0])
    assert b4["roots"][0] >= 0
    leaves4, depth4, seen = _walk4(b4["nodes"], b4["roots"][0], b4["leaf_base"][0])
    assert len(seen) == len(b4["nodes"])          # no orphan nodes
    key = lambda lv: (lv[0], lv[1], lv[2][0].tobytes(), lv[2][1].tobytes())
    assert sorted(map(key, leaves4)) == sorted(map(key, leaves2))
    assert depth4 <= depth2 and len(b4["nodes"]) <= len(b["nodes"])
    assert max(c for _, c, _ in leaves4) <= 31


def test_bvh4_roots_for_every_mesh_of_the_reference_scene(pt_mod):
    s = pt_mod.Scene(REF_SCENE)
    s.build(bvh=True)
    b4 = s.export_bvh4()
    assert (b4["roots"] >= 0).all() and len(b4["nodes"]) > 0


def _tiny_mesh(n):
    """n disjoint triangles (n = 0: a mesh with no triangles)."""
    pos = np.zeros((3 * n, 3), np.float32)
    for i in range(n):
        pos[3 * i:3 * i + 3] = np.float32([[i, 0, 0], [i + 0.5, 0, 0], [i, 0.5, 0.2]])
    nrm = np.tile(np.float32([0, 0, 1]), (3 * n, 1))
    return pos, nrm, np.arange(3 * n, dtype=np.int32).reshape(-1, 3)


@pytest.mark.parametrize("ntri", [1, 2, 3, 10, 5000])
def test_bvh4_empty_slots_are_inverted_infinite_boxes(pt_mod, ntri):
    """The node steps never read Bvh4Node.count: an empty slot must miss the
    near / far slab test by itself, which the inverted infinite box
    (lo = +inf, hi = -inf) guarantees for every ray (entry +inf, exit -inf),
    with link -1.  That holds for slots past the children and for an empty
    binary child (a 1- or 2-triangle mesh: a root leaf beside an empty child).
    Every other slot's box is finite and ordered."""
    from pathtracerap_amd.synthetic import torus_mesh
    pos, nrm, tris = torus_mesh(ntri, seed=2) if ntri >= 10 else _tiny_mesh(ntri)
    s = pt_mod.Scene()
    m = s.addMesh(pos, nrm, tris)
    s.addModel(m, (1, 1, 1), (0, 0, 0), (0, 0, 0), "DIFFUSE", (1, 1, 1))
    s.build(bvh=True)
    b4 = s.export_bvh4()
    nodes = b4["nodes"]
    assert b4["roots"][0] >= 0 and len(nodes) > 0
    ints = nodes.view(np.int32)
    empty = ints[:, 28:32] < 0
    lo = np.stack([nodes[:, 0:4], nodes[:, 4:8], nodes[:, 8:12]])
    hi = np.stack([nodes[:, 12:16], nodes[:, 16:20], nodes[:, 20:24]])
    assert empty.any() or ntri > 10       # a small mesh leaves slots empty
    assert (lo[:, empty] == np.inf).all() and (hi[:, empty] == -np.inf).all()
    assert (ints[:, 24:28][empty] == -1).all() and (ints[:, 28:32][empty] == -1).all()
    full = ~empty
    assert np.isfinite(lo[:, full]).all() and np.isfinite(hi[:, full]).all()
    assert (lo[:, full] <= hi[:, full]).all()
    leaves, _, _ = _walk4(nodes, b4["roots"][0], b4["leaf_base"][0])
    assert sum(c for _, c, _ in leaves) == len(tris)


def test_bvh4_leaf_links_are_relative_to_their_mesh(pt_mod):
    """A 4-wide leaf link holds its first record relative to the mesh's
    leaf_base (ModelRec::leaf_base, added back by the traces), so the 2^26
    limit of the stack's leaf encoding applies per mesh: every mesh's
    smallest relative first is 0, and leaf_base + first gives exactly the
    binary BLAS's leaves of that mesh, whatever precedes it in bvh_tri_order."""
    from pathtracerap_amd.synthetic import torus_mesh
    s = pt_mod.Scene()
    sizes = [5000, 1, 300, 2, 12000]
    for i, n in enumerate(sizes):
        pos, nrm, tris = torus_mesh(n, seed=5 + i) if n >= 10 else _tiny_mesh(n)
        m = s.addMesh(pos + np.float32(3 * i), nrm, tris)
        s.addModel(m, (1, 1, 1), (0, 0, 0), (0, 0, 0), "DIFFUSE", (1, 1, 1))
        sizes[i] = len(tris)
    s.build(bvh=True)
    b, b4 = s.export_bvh(), s.export_bvh4()
    assert (b4["roots"] >= 0).all()
    assert b4["leaf_base"][0] == 0 and (np.diff(b4["leaf_base"]) > 0).all()
    key = lambda lv: (lv[0], lv[1], lv[2][0].tobytes(), lv[2][1].tobytes())
    for mi, n in enumerate(sizes):
        rel, _, _ = _walk4(b4["nodes"], b4["roots"][mi])
        assert min(f for f, _, _ in rel) == 0
        abs4, _, _ = _walk4(b4["nodes"], b4["roots"][mi], b4["leaf_base"][mi])
        leaves2, _ = _walk(b["nodes"], b["roots"][mi])
        assert sorted(map(key, abs4)) == sorted(map(key, leaves2))
        assert sum(c for _, c, _ in abs4) == n
