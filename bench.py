#!/usr/bin/env python3
"""Benchmark: Mrays/s of the MI355X bounce loop on BASELINE.json configs[1].

    python bench.py [--gpus N] [--steps K] [--warmup W] [--accel bvh|grid]

Default mode ``grid_fast`` returns the reference algorithm's results bit for
bit (uniform-grid semantics computed through a BVH hit set); the exact
closest-hit ``bvh`` mode is timed after it and reported under ``alt_mode``.

Workload (configs[1]): diffuse-only synthetic OBJ (~100k triangles, a
displaced torus in an open-front room with emissive panels), 1280x1024,
8 bounces.  One step = one sample per pixel = one full pass of the bounce
loop (camera rays from the primary-hit cache, intersect, scatter, compact,
accumulate) over the whole frame; the scene, ray pools and accumulator are
resident in HBM before the timed region starts.

Multi-GPU (``torchrun --nproc-per-node N bench.py --gpus N``): samples shard
across ranks (rank r renders iterations [r*K, (r+1)*K)), then one RCCL
all-reduce sums the float3 accumulator; weak scaling.

Prints ONE JSON line (rank 0).  ``value`` = ray segments shaded per second
over all ranks (a segment = one live ray in one bounce, primary rays
included) in millions; ``samples_per_sec`` = pixel samples per second.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mrays/sec + samples/sec at 1280×1024, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--accel", choices=["bvh", "grid", "grid_fast"], default="grid_fast",
                    help="grid_fast: the reference's grid results (bit-identical), BVH-accelerated; "
                         "bvh: exact closest hit; grid: the reference's list-walking DDA")
    ap.add_argument("--alt-accel", default="bvh", help="second mode timed after the main one ('' to skip)")
    ap.add_argument("--ntri", type=int, default=100_000)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=1024)
    ap.add_argument("--bounces", type=int, default=8)
    ap.add_argument("--metallic", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU baseline duration")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-kernel HIP-event pass")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="process group for N>1 (nccl = RCCL over xGMI; gloo only to rehearse the "
                         "multi-rank path with several ranks on one GPU)")
    ap.add_argument("--pipelines", type=int, default=16,
                    help="iterations in flight on their own HIP streams (0: the library default, 8)")
    ap.add_argument("--hw-queues", type=int, default=16,
                    help="GPU_MAX_HW_QUEUES for this process (HIP default 4): one hardware queue per "
                         "pipeline stream so iterations in flight do not serialise on a shared queue (max 32)")
    return ap.parse_args()


def cpu_baseline(scene_path, accel_name, bounces, width, height, target_s):
    """The oracle (C port of the reference's bounce loop) on the host cores:
    same scene and camera, reduced resolution, 1 sample per pixel, sized to
    about ``target_s`` seconds of CPU work."""
    import oracle as O
    import pathtracerap_amd as P
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import flat_from_export

    threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 1))
    s = P.Scene(scene_path)
    s.build()
    flat = flat_from_export(s.export())

    def run(w, h, iters):
        cfg = O.RenderConfig(width=w, height=h, iterations=iters, max_bounces=bounces, accel=0, threads=threads)
        t = time.perf_counter()
        _, seg = O.render(flat, cfg)
        return seg, time.perf_counter() - t

    # probe on a 1/16-pixel frame, then size the real sample to ~target_s
    w, h, iters = max(8, width // 4), max(8, height // 4), 1
    seg, dt = run(w, h, iters)
    frames = target_s / max(dt, 1e-3)          # probe-frames that fit the budget
    if frames >= 16:
        w, h, iters = width, height, max(1, int(frames / 16))
    else:
        f = max(1.0, frames) ** 0.5
        w, h = min(width, int(w * f)), min(height, int(h * f))
    seg, dt = run(w, h, iters)
    return {"value": seg / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"oracle/ptoracle.c (C port of the reference renderLoop, uniform-grid accel as in "
                      f"the reference) on the same scene/camera at {w}x{h}, {iters} spp, {bounces} bounces: "
                      f"{seg} segments in {dt:.2f}s on {threads} thread(s)"}


def workload_name(args):
    """Label of the BASELINE.json configuration this run measures."""
    default = (args.ntri == 100_000 and args.width == 1280 and args.height == 1024 and args.bounces == 8
               and not args.metallic)
    if default:
        return "configs[1]: diffuse-only synthetic OBJ (~100k tris), 1280x1024, 8 bounces"
    kind = "metallic+diffuse" if args.metallic else "diffuse-only"
    tag = {(True, 2800): "configs[2] shape: ", (False, 1280): ""}.get((args.metallic, args.width), "")
    if not args.metallic and args.ntri >= 5_000_000:
        tag = "configs[4] shape: "
    elif not args.metallic and args.ntri >= 500_000:
        tag = "north_star target shape: "
    return f"{tag}{kind} synthetic OBJ (~{args.ntri} tris), {args.width}x{args.height}, {args.bounces} bounces"


def load_pmc(kernel, workload_key):
    """HBM bytes per launch of ``kernel`` from the committed rocprofv3 PMC
    summary (scripts/pmc_summary.py), corrected per MI355X_MICROARCH.md
    (FETCH_SIZE x2 on gfx950, KB -> bytes); None when absent."""
    path = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(workload_key, {}).get(kernel)
        return None if e is None else e["hbm_bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        return None


VALU_PEAK_G = 256 * 4 * 2.4 / 2   # G wave-instructions/s: 1024 SIMDs, one wave64 VALU op per 2 cycles at 2.4 GHz


def load_sq(workload_key, tag="_sq"):
    """VALU / SALU wave-instruction counts of the committed rocprofv3
    SQ_INSTS_VALU / SQ_INSTS_SALU pass (scripts/pmc_summary.py sq): tag "_sq" with
    the bench's pipelines, "_sq_p1" with one pipeline; None when absent."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_latest.json")) as f:
            return json.load(f).get(workload_key, {}).get(tag)
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    if args.hw_queues > 0:     # read once by the HIP runtime at initialisation: set before torch touches it
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, args.hw_queues))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one rank per GPU; with fewer GPUs than ranks (a gloo rehearsal on a 1-GPU
    # box) ranks share devices round-robin
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import pathtracerap_amd as P
    from pathtracerap_amd import synthetic

    tmp = tempfile.mkdtemp(prefix=f"ptbench_r{rank}_")
    scene_path = synthetic.diffuse_scene(tmp, ntri=args.ntri, width=args.width, height=args.height,
                                         bounces=args.bounces, accel=args.accel, metallic=args.metallic)
    accel = {"bvh": P.ACCEL_BVH, "grid": P.ACCEL_GRID, "grid_fast": P.ACCEL_GRID_FAST}[args.accel]
    scene = P.Scene(scene_path)
    cfg = scene.apply_settings(P.RenderConfig())
    cfg.width, cfg.height, cfg.max_bounces, cfg.accel = args.width, args.height, args.bounces, accel
    if args.pipelines > 0:
        cfg.pipelines = args.pipelines
    scene.build(grid=cfg.grid, bvh=accel != P.ACCEL_GRID)
    ntri = scene.counts()["nt"]

    image = torch.zeros(cfg.width * cfg.height * 3, dtype=torch.float32, device=dev)
    r = P.Renderer(cfg)
    r.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    r.bind_image(image.data_ptr(), keepalive=image)
    r.allocateOnGPU(scene)

    K, W = args.steps, args.warmup
    # warmup: builds the primary-hit cache, warms caches/clocks; distinct iteration ids
    r.renderLoop(first_iter=1_000_000 + rank * max(W, 1), n_iters=W, sync=False)
    torch.cuda.synchronize(dev)
    if world > 1:
        # warm the accumulator-sized all-reduce too: any one-time RCCL setup for a
        # message of this size is paid here, not inside the timed region
        dist.all_reduce(image, op=dist.ReduceOp.SUM)
        torch.cuda.synchronize(dev)
    r.clearImage()
    seg0 = r.segments()
    pb0 = r.segments_per_bounce()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    r.renderLoop(first_iter=rank * K, n_iters=K, sync=False)
    if world > 1:
        dist.all_reduce(image, op=dist.ReduceOp.SUM)      # RCCL over xGMI
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()

    seg = r.segments() - seg0
    faults = r.trace_faults()
    if faults:   # a persistent trace gave up: rays kept stale hits, the measured image is wrong
        raise SystemExit(f"bench: {faults} persistent-trace wave(s) hit the iteration cap; result invalid")
    per_bounce = [a - b for a, b in zip(r.segments_per_bounce(), pb0)]
    while per_bounce and per_bounce[-1] == 0:
        per_bounce.pop()
    workload_key = f"{args.accel}_{args.ntri}_{args.width}x{args.height}_b{args.bounces}" + ("_metal" if args.metallic else "")
    elapsed = t1 - t0
    t = torch.tensor([elapsed, float(seg)], dtype=torch.float64, device=dev)
    if world > 1:
        tmax = t[0:1].clone(); dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t[1:2].clone(); dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed, seg_total = float(tmax.item()), float(tsum.item())
    else:
        seg_total = float(seg)
    img_ok = bool(torch.isfinite(image).all().item())
    pipes = r.pipelines()
    r.free()

    # Per-kernel durations for the roofline come from a separate pass of the
    # same K iterations with ONE pipeline: with several iterations in flight
    # the kernels of different pipelines overlap and an event pair around one
    # launch would also time its neighbours.  Same iteration ids => the same
    # per-bounce ray counts as the timed pass.
    stats = None
    if not args.no_profile and rank == 0:
        cfg_p = P.RenderConfig(**{**cfg.__dict__, "pipelines": 1})
        rp = P.Renderer(cfg_p)
        rp.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        rp.bind_image(image.data_ptr(), keepalive=image)
        rp.allocateOnGPU(scene)
        rp.renderLoop(first_iter=1_000_000, n_iters=W, sync=False)
        torch.cuda.synchronize(dev)
        rp.kernel_stats()          # reset
        rp.set_profiling(True)
        rp.renderLoop(first_iter=rank * K, n_iters=K, sync=True)
        stats = rp.kernel_stats()
        rp.free()

    alt = None
    if args.alt_accel and args.alt_accel != args.accel:
        acc2 = {"bvh": P.ACCEL_BVH, "grid": P.ACCEL_GRID, "grid_fast": P.ACCEL_GRID_FAST}[args.alt_accel]
        cfg2 = P.RenderConfig(width=cfg.width, height=cfg.height, max_bounces=cfg.max_bounces, accel=acc2,
                              grid=cfg.grid, block=cfg.block, pipelines=cfg.pipelines)
        if acc2 != P.ACCEL_GRID and accel == P.ACCEL_GRID:
            scene.build(grid=cfg.grid, bvh=True)
        r2 = P.Renderer(cfg2)
        r2.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        r2.bind_image(image.data_ptr(), keepalive=image)
        r2.allocateOnGPU(scene)
        r2.renderLoop(first_iter=2_000_000 + rank * max(W, 1), n_iters=W, sync=False)
        torch.cuda.synchronize(dev)
        s2 = r2.segments()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        a0 = time.perf_counter()
        r2.renderLoop(first_iter=rank * K, n_iters=K, sync=False)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        a1 = time.perf_counter()
        seg2 = float(r2.segments() - s2)
        if r2.trace_faults():
            raise SystemExit(f"bench: alt mode {args.alt_accel}: persistent trace hit the iteration cap")
        r2.free()
        ta = torch.tensor([a1 - a0, seg2], dtype=torch.float64, device=dev)
        if world > 1:
            tm = ta[0:1].clone(); dist.all_reduce(tm, op=dist.ReduceOp.MAX)
            ts = ta[1:2].clone(); dist.all_reduce(ts, op=dist.ReduceOp.SUM)
            ta = torch.cat([tm, ts])
        alt = {"accel": args.alt_accel, "value": round(float(ta[1]) / float(ta[0]) / 1e6, 3), "unit": "Mrays/s",
               "ms_per_step": round(float(ta[0]) / K * 1e3, 3),
               "samples_per_sec": round(world * K * cfg.width * cfg.height / float(ta[0]), 1),
               "semantics": "exact closest hit (statistically equivalent image, not per-pixel identical)"
               if args.alt_accel == "bvh" else "reference grid (bit-identical)"}

    if rank == 0:
        npix = cfg.width * cfg.height
        mrays = seg_total / elapsed / 1e6
        samples = world * K * npix / elapsed
        roof = None
        if stats and stats["bounce_ms"] > 0:
            # Dominant kernel on bounces >= 1 (see DESIGN.md "Kernels and their rooflines").
            # Fused k_bounce: per ray segment entering bounce b >= 1, 48 B ray-state gather; a
            # survivor writes 48 B of compacted state, a terminated ray read-modify-writes its
            # 12 B accumulator pixel.  Split path (ACCEL_BVH): k_trace_bvh reads o, d (32 B) and
            # writes the 20 B hit record per segment; the shading pass reads ray + hit (68 B)
            # and writes as above.  Scene data (BVH nodes / triangles) is cache-resident and not
            # counted.
            nb = [x for x in per_bounce]
            shade_bytes = 0.0
            trace_bytes = 0.0
            split = stats.get("trace_launches", 0) > 0
            for b in range(1, len(nb)):
                nxt = nb[b + 1] if b + 1 < len(nb) else 0
                shade_bytes += (68.0 if split else 48.0) * nb[b] + 48.0 * nxt + 24.0 * (nb[b] - nxt)
                trace_bytes += 52.0 * nb[b]
            shade = {"launches": stats["bounce_launches"],
                     "avg_launch_ms": round(stats["bounce_ms"] / max(stats["bounce_launches"], 1), 4)}
            if split:
                kname = "k_trace_bvh" if args.accel == "bvh" else "k_trace_gf"
                nbytes, kms, launches = trace_bytes, stats["trace_ms"], max(stats["trace_launches"], 1)
                shade["kernel"] = "k_bounce<false,hitbuf>"
                shade["achieved_gbs"] = round(shade_bytes / (stats["bounce_ms"] / 1e3) / 1e9, 2)
            else:
                kname = f"k_bounce<false,{args.accel}>"
                nbytes, kms, launches = shade_bytes, stats["bounce_ms"], max(stats["bounce_launches"], 1)
                shade = None
            achieved = nbytes / (kms / 1e3) / 1e9
            traffic = load_pmc(kname, workload_key)
            roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                    "kernel": kname, "algorithmic_bytes_per_launch": round(nbytes / launches),
                    "avg_launch_ms": round(kms / launches, 4), "launches": launches,
                    "shading_pass": shade,
                    "first_bounce_avg_ms": round(stats["first_ms"] / max(stats["first_launches"], 1), 4),
                    "scan_avg_ms": round(stats["scan_ms"] / max(stats["scan_launches"], 1), 4)}
        # Issue roofline: the traces are bound by instruction issue and dependent-load
        # latency, not by HBM bytes, so the VALU issue rate against the SIMDs' peak is
        # the informative fraction -- for the whole job (all kernels of a step, with the
        # pipelines overlapping) and for the dominant kernel's single-pipeline launches.
        issue = None
        sq = load_sq(workload_key)
        if sq:
            v_step = sq["valu_insts_per_iteration"]
            job = v_step * K / elapsed / 1e9          # per GPU: each rank runs K steps in `elapsed`
            issue = {"bound": "valu", "unit": "G wave-instr/s", "peak": VALU_PEAK_G,
                     "job": {"valu_insts_per_step": round(v_step), "achieved": round(job, 1),
                             "frac": round(job / VALU_PEAK_G, 4),
                             "salu_insts_per_step": round(sq["salu_insts_per_iteration"]),
                             "salu_achieved": round(sq["salu_insts_per_iteration"] * K / elapsed / 1e9, 1)},
                     "source": "rocprofv3 SQ_INSTS_VALU / SQ_INSTS_SALU pass (profiles/pmc_latest.json)"}
            sq1 = load_sq(workload_key, "_sq_p1")     # the roofline pass runs one pipeline
            kk = sq1["kernels"].get(roof["kernel"]) if (roof and sq1) else None
            if kk:
                ach = kk["valu_insts_per_launch"] / (roof["avg_launch_ms"] / 1e3) / 1e9
                issue["kernel"] = {"name": roof["kernel"], "valu_insts_per_launch": round(kk["valu_insts_per_launch"]),
                                   "avg_launch_ms": roof["avg_launch_ms"], "achieved": round(ach, 1),
                                   "frac": round(ach / VALU_PEAK_G, 4)}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(scene_path, args.accel, args.bounces, cfg.width, cfg.height, args.cpu_seconds)
            except Exception as e:  # noqa: BLE001 -- reported, not fatal
                cpu = {"error": repr(e)}
        out = {
            "metric": METRIC, "value": round(mrays, 3), "unit": "Mrays/s", "n_gpus": world, "steps": K,
            "warmup": W, "ms_per_step": round(elapsed / K * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "samples_per_sec": round(samples, 1),
            "config": {"workload": workload_name(args),
                       "triangles": ntri, "width": cfg.width, "height": cfg.height, "bounces": cfg.max_bounces,
                       "spp_per_step": 1, "accel": args.accel,
                       "results": "bit-identical to the reference algorithm (oracle-checked)"
                       if args.accel != "bvh" else "exact closest hit",
                       "parallelism": f"samples sharded x{world}" + (" (gloo rehearsal)" if world > 1 and args.dist_backend == "gloo" else ""), "pipelines": pipes,
                       "segments": int(seg_total), "segments_per_bounce_rank0": per_bounce,
                       "image_finite": img_ok, "trace_faults": faults},
            "roofline": roof, "issue_roofline": issue, "cpu_baseline": cpu, "alt_mode": alt,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
