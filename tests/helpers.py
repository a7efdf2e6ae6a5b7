"""Shared helpers for the parity tests (test infrastructure)."""
import numpy as np

import oracle as O


def flat_from_export(a: dict, gdim=(25, 25, 25)) -> "O.FlatScene":
    return O.FlatScene(vpos=a["vpos"], vnrm=a["vnrm"], tris=a["tris"], mesh_ranges=a["mesh_ranges"],
                       mesh_bbox=a["mesh_bbox"], model_ints=a["model_ints"], model_m2w=a["model_m2w"],
                       model_w2m=a["model_w2m"], model_color=a["model_color"], grid_ints=a["grid_ints"],
                       grid_vw=a["grid_vw"], vox=a["vox"], per_voxel=a["per_voxel"], gdim=tuple(gdim))


def oracle_cfg(cfg, threads=1) -> "O.RenderConfig":
    return O.RenderConfig(width=cfg.width, height=cfg.height, iterations=cfg.iterations, first_iter=0,
                          max_bounces=cfg.max_bounces, accel=oracle_accel(cfg.accel), threads=threads, tail_drop=cfg.tail_drop,
                          cam=tuple(cfg.cam), plane_z=cfg.plane_z, plane_x0=cfg.plane_x0, plane_y0=cfg.plane_y0,
                          plane_w=cfg.plane_w, plane_h=cfg.plane_h)


def oracle_accel(accel):
    """GPU accel -> oracle semantics: GRID (0) and GRID_FAST (2) are the
    reference grid; BVH (1) is the exact closest hit."""
    return 1 if accel == 1 else 0


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


def assert_bitexact(got, want, what):
    got = np.asarray(got); want = np.asarray(want)
    assert got.shape == want.shape, (what, got.shape, want.shape)
    g, w = bits(got), bits(want)
    bad = np.nonzero(g.reshape(-1) != w.reshape(-1))[0]
    if len(bad):
        i = bad[0]
        raise AssertionError(f"{what}: {len(bad)} of {g.size} elements differ; first at flat {i}: "
                             f"got {got.reshape(-1)[i]!r} want {want.reshape(-1)[i]!r}")
