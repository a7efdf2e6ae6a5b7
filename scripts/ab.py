#!/usr/bin/env python3
"""In-process A/B of renderer variants on the bench workload (interleaved
rounds on one device; cdna_hip_programming.md §5.4 rule 24).

    python scripts/ab.py --variants bvh:256 bvh:128 bvh:64 grid:256 --rounds 5 --steps 8
    python scripts/ab.py --variants bvh:64:PT_TRACE_SPLIT=0 bvh:64:PT_TRACE_REFILL=8   (env read at allocateOnGPU)
"""
import argparse
import json
import os
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="+", default=["bvh:256", "bvh:128", "bvh:64"])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--ntri", type=int, default=100_000)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=1024)
    ap.add_argument("--bounces", type=int, default=8)
    ap.add_argument("--scene", default=None, help="scene file instead of the synthetic one")
    ap.add_argument("--inmem", action="store_true", help="the synthetic scene built in memory (no OBJ text: 10M triangles)")
    a = ap.parse_args()
    import torch
    import pathtracerap_amd as P
    from pathtracerap_amd import synthetic
    path = a.scene or (None if a.inmem else synthetic.diffuse_scene(tempfile.mkdtemp(), ntri=a.ntri))
    scenes = {}
    rs = {}
    for v in a.variants:
        parts = v.split(":")
        accel, block = parts[0], parts[1]
        env = dict(kv.split("=") for kv in parts[2].split(",")) if len(parts) > 2 else {}
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)          # read by allocateOnGPU
        acc = {"bvh": P.ACCEL_BVH, "grid": P.ACCEL_GRID, "grid_fast": P.ACCEL_GRID_FAST}[accel]
        # build-time variables (PT_BVH*: read by Scene::build) get a scene of their own
        skey = (acc, tuple(sorted((k, v) for k, v in env.items() if k.startswith("PT_BVH"))))
        if skey not in scenes:
            if a.inmem and not a.scene:
                s = synthetic.build_scene(P, ntri=a.ntri)
            else:
                s = P.Scene(path)
                s.build(bvh=acc != P.ACCEL_GRID)
            scenes[skey] = s
        cfg = P.RenderConfig(width=a.width, height=a.height, max_bounces=a.bounces, accel=acc, block=int(block))
        r = P.Renderer(cfg)
        r.allocateOnGPU(scenes[skey])
        for k, old in saved.items():
            if old is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = old
        r.renderLoop(1000, 2)          # warm + primary cache
        rs[v] = r
    times = {v: [] for v in a.variants}
    segs = {}
    dfr = {v: 0 for v in a.variants}
    for rnd in range(a.rounds):
        for v, r in rs.items():
            s0 = r.segments()
            d0 = r.deferred_rays()
            torch.cuda.synchronize()
            t = time.perf_counter()
            r.renderLoop(rnd * a.steps, a.steps)
            times[v].append((time.perf_counter() - t) / a.steps * 1e3)
            segs[v] = (r.segments() - s0) / a.steps
            dfr[v] += r.deferred_rays() - d0
    out = {}
    for v in a.variants:
        med = statistics.median(times[v])
        out[v] = {"ms_per_spp_median": round(med, 3), "ms_min": round(min(times[v]), 3),
                  "Mrays_s": round(segs[v] / med / 1e3, 1)}
        if dfr[v]:                                     # rays k_trace_deferred traced (hit-set pool exhausted / full)
            out[v]["deferred_rays_per_spp"] = round(dfr[v] / (a.rounds * a.steps), 1)
        allc = rs[v].segments_per_bounce(159)
        if allc[71]:
            it = allc[71]
            out[v]["trace_iters_per_wave_total"] = it
            ph = {k: (allc[i + 7], allc[i]) for k, i in
                  (("node", 72), ("leaf", 73), ("walk", 74), ("select", 75))}
            out[v]["phase_iters"] = {k: a for k, (a, b) in ph.items()}
            out[v]["lanes_per_phase_iter"] = {k: round(b / max(a, 1), 2) for k, (a, b) in ph.items()}
            out[v]["select_loop_trips"] = allc[76]
            out[v]["deferred"] = allc[77]
            sg = max(rs[v].segments(), 1)
            out[v]["wave_iters_per_segment"] = round(it / sg, 3)
            # diagnostic slot S lives at segments[S + 64] = allc[S + 63]
            out[v]["busy_lanes_per_iter"] = round(allc[109] / it, 2)
            out[v]["drain_iter_share"] = round(allc[107] / it, 3)
            out[v]["busy_lanes_per_drain_iter"] = round(allc[108] / max(allc[107], 1), 2)
            out[v]["phase_iters_per_segment"] = {k: round(a / sg, 3) for k, (a, b) in ph.items()}
            out[v]["tail_iter_share"] = round(allc[78] / it, 3)          # slot 15: tail launches' wave-iterations
            out[v]["busy_lanes_per_tail_iter"] = round(allc[106] / max(allc[78], 1), 2)   # slot 43
        if allc[129]:                                  # slots 64..68 (stats build, & 16): 4-wide node steps
            sg = max(rs[v].segments(), 1)
            out[v]["node4"] = {"visits_per_segment": round(allc[129] / sg, 2),
                               "hit_children_per_visit": round(allc[130] / allc[129], 3),
                               "pushes_per_visit": round(allc[127] / allc[129], 3),
                               "spilled_push_share": round(allc[128] / max(allc[127], 1), 4),
                               "tri_tests_per_segment": round(allc[131] / sg, 2)}
        if any(allc[110:114]):                         # slots 47..50 (k_scan, stats build): hand-on volume
            sg = max(rs[v].segments(), 1)
            out[v]["handons_per_segment"] = dict(zip(["drained_l0", "walk_handons", "deferred", "drained_l1"],
                                                     [round(c / sg, 5) for c in allc[110:114]]))
        if "PT_DEBUG_ABLATE=32" in v or "PT_DEBUG_ABLATE=96" in v:   # cycle stamps
            cyc = allc[83:89]
            tot = max(sum(cyc), 1)
            out[v]["cycle_share"] = dict(zip(["refill", "select", "leaf", "node", "walk", "handon_drain"],
                                             [round(c / tot, 3) for c in cyc]))
            tc = allc[133:139]                       # slots 70..75: the tail launches' cycles by phase
            if any(tc):
                out[v]["tail_cycle_share_of_all"] = round(sum(tc) / tot, 3)
                out[v]["tail_cycle_share"] = dict(zip(["resume", "select", "leaf", "node", "walk", "handon_drain"],
                                                      [round(c / sum(tc), 3) for c in tc]))
            rr = allc[118:122]                       # slots 55..58: refill claim / order+gather / -, pre-refill
            out[v]["refill_split_share"] = dict(zip(["claim", "-", "order_and_gather", "stores_before"],
                                                    [round(c / tot, 3) for c in rr]))
            out[v]["handon_iters_per_segment"] = round(allc[89] / max(rs[v].segments(), 1), 5)
            out[v]["drains_per_segment"] = round(allc[90] / max(rs[v].segments(), 1), 5)
            out[v]["wave_cycles_per_segment"] = round(tot / max(rs[v].segments(), 1), 1)
        if "PT_DEBUG_ABLATE=96" in v:
            w3 = allc[92:95]
            out[v]["walk_wave_cycles_per_segment"] = dict(zip(["init_union", "skip", "steps"],
                                                              [round(c / max(rs[v].segments(), 1), 1) for c in w3]))
        elif allc[84]:                                 # PT_TRACE_STATS build, PT_DEBUG_ABLATE & 4
            segs_all = rs[v].segments()
            out[v]["walk_steps_per_walk"] = round(allc[83] / allc[84], 2)
            out[v]["walks_per_segment"] = round(allc[84] / segs_all, 3)
            out[v]["members_per_walk"] = round(allc[87] / allc[84], 2)
            out[v]["walk_steps_per_segment_by_model"] = [round(x / segs_all, 2) for x in allc[88:92]]
        if allc[86]:
            out[v]["collect_nodes_per_collection"] = round(allc[85] / allc[86], 2)
            out[v]["collections_per_segment"] = round(allc[86] / rs[v].segments(), 3)
        if any(allc[143:151]):                         # slots 80..87: the fast certificate's first failed condition
            tot = max(sum(allc[143:151]), 1)
            out[v]["cert_fast_fail_share"] = dict(zip(
                ["ties_or_none", "zero_dir", "thin_box", "misses_Bstar", "grazes_Bstar", "window",
                 "member_one_extension", "member_several_extensions"], [round(c / tot, 4) for c in allc[143:151]]))
        if allc[105]:                                  # slots 40..42: fast / full certificate outcomes
            out[v]["cert_attempts_per_segment"] = round(allc[105] / max(rs[v].segments(), 1), 5)
            out[v]["cert_fast_ok_share"] = round(allc[103] / allc[105], 4)
            out[v]["cert_full_ok_after_fast_share"] = round(allc[104] / allc[105], 4)
        cf = allc[95:103]
        if any(cf):
            out[v]["cert_fail_per_segment"] = dict(zip(["ties", "zero_dir", "start_shift", "starts_in_U", "grazes_U",
                                                        "margin", "not_in_Bstar", "window"],
                                                       [round(c / max(rs[v].segments(), 1), 4) for c in cf]))
            out[v]["cert_ok_per_segment"] = round(allc[76] / max(rs[v].segments(), 1), 4)
        wb = allc[114:118]                             # slots 51..54: walks by hit-set size 1, 2, 3, >= 4
        if any(wb):
            out[v]["walks_by_hitset_size"] = dict(zip(["1", "2", "3", ">=4"], [round(c / max(sum(wb), 1), 3) for c in wb]))
        diag = allc[64:67]
        if any(diag):
            out[v]["diag_tier2_t1overflow_fallback"] = diag
        if allc[69]:
            out[v]["nodes_per_traversal"] = round(allc[67] / allc[69], 2)
            out[v]["tris_per_traversal"] = round(allc[68] / allc[69], 2)
            out[v]["traversals_per_segment"] = round(allc[69] / rs[v].segments(), 3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
