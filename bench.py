#!/usr/bin/env python3
"""Benchmark: Mrays/s of the MI355X bounce loop on BASELINE.json configs[1].

    python bench.py [--gpus N] [--steps K] [--warmup W] [--accel bvh|grid|grid_fast]

Default mode ``grid_fast`` returns the reference algorithm's results bit for
bit (uniform-grid semantics computed through a BVH hit set); the exact
closest-hit ``bvh`` mode is timed after it and reported under ``alt_mode``.

Workload (configs[1]): diffuse-only synthetic OBJ (~100k triangles, a
displaced torus in an open-front room with emissive panels), 1280x1024,
8 bounces.  One step = one sample per pixel = one full pass of the bounce
loop (camera rays from the primary-hit cache, intersect, scatter, compact,
accumulate) over the whole frame; the scene, ray pools and accumulator are
resident in HBM before the timed region starts.  ``targets`` times two more
workloads the same way: north_star's target (the 1M-triangle diffuse OBJ at
1280x1024) and configs[2] (the README render's own scene, Scene.cpp:3-224,
at 2800x2240).

Multi-GPU (``torchrun --nproc-per-node N bench.py --gpus N``): samples shard
across ranks (rank r renders iterations [r*K, (r+1)*K)), then one RCCL
all-reduce sums the float3 accumulator; weak scaling.

Prints ONE JSON line (rank 0).  ``value`` = ray segments shaded per second
over all ranks (a segment = one live ray in one bounce, the primary rays whose
hits come from the first-intersection cache included, as the reference counts
its loop's work) in millions; ``traced_mrays_per_sec`` leaves the cached
primary segments out; ``samples_per_sec`` = pixel samples per second.
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
# G wave-instructions/s: 256 CUs x 4 SIMDs, one wave64 VALU instruction per SIMD every
# 2 cycles (32 lanes/cycle, MI355X_MICROARCH.md:54 and its constants table, v_fma_f32
# "2 cyc (SIMD-32)"), 2.4 GHz
VALU_PEAK_G = 256 * 4 * 2.4 / 2


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
    ap.add_argument("--scene", default="", help="a scene file instead of the synthetic OBJ scene (e.g. "
                                                "scenes/reference_scene.txt); its RENDER block's bounces apply")
    ap.add_argument("--targets", default="target_1m,configs2",
                    help="extra workloads timed after the main line ('' to skip): target_1m = north_star's "
                         "1M-triangle scene at 1280x1024; configs2 = the README scene at 2800x2240")
    ap.add_argument("--target-steps", type=int, default=16)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU baseline duration")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="no per-kernel HIP events (neither in the timed "
                                                              "region nor the one-pipeline pass)")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="process group for N>1 (nccl = RCCL over xGMI; gloo only to rehearse the "
                         "multi-rank path with several ranks on one GPU)")
    ap.add_argument("--pipelines", type=int, default=16,
                    help="iterations in flight on their own HIP streams (0: the library default, 16)")
    ap.add_argument("--hw-queues", type=int, default=16,
                    help="GPU_MAX_HW_QUEUES for this process (HIP default 4; the library also defaults it "
                         "to 16): one hardware queue per pipeline stream (max 32)")
    return ap.parse_args()


def cpu_baseline(scene_path, bounces, width, height, target_s):
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
    if args.scene:
        return f"scene file {os.path.relpath(args.scene, ROOT)}, {args.width}x{args.height}, {args.bounces} bounces"
    default = (args.ntri == 100_000 and args.width == 1280 and args.height == 1024 and args.bounces == 8
               and not args.metallic)
    if default:
        return "configs[1]: diffuse-only synthetic OBJ (~100k tris), 1280x1024, 8 bounces"
    kind = "metallic+diffuse" if args.metallic else "diffuse-only"
    tag = ""
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


def load_sq(workload_key, tag="_sq"):
    """VALU / SALU wave-instruction counts of the committed rocprofv3
    SQ_INSTS_VALU / SQ_INSTS_SALU pass (scripts/pmc_summary.py sq): tag "_sq" with
    the bench's pipelines, "_sq_p1" with one pipeline; None when absent."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_latest.json")) as f:
            return json.load(f).get(workload_key, {}).get(tag)
    except (OSError, ValueError):
        return None


class Ctx:
    """Process-group plumbing shared by every timed workload."""

    def __init__(self, torch, dist, dev, rank, world):
        self.torch, self.dist, self.dev, self.rank, self.world = torch, dist, dev, rank, world

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def reduce(self, vals, op):
        """vals (floats) reduced over ranks with op ('max' / 'sum')."""
        t = self.torch.tensor(vals, dtype=self.torch.float64, device=self.dev)
        if self.world > 1:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM)
        return [float(x) for x in t.cpu()]


def timed_run(P, ctx, scene, cfg, K, W, iter_base, events, reduce_image):
    """Warm up, then time exactly K iterations (this rank's [rank*K, (rank+1)*K))
    between barrier + synchronize pairs; the accumulator all-reduce (RCCL) is
    inside the timed region.  ``events``: per-kernel HIP events on the pipeline
    streams during the timed region (renderer profiling mode).  Returns the
    max-over-ranks time, the all-rank segment total and the renderer's stats."""
    torch, dev, rank = ctx.torch, ctx.dev, ctx.rank
    image = torch.zeros(cfg.width * cfg.height * 3, dtype=torch.float32, device=dev)
    r = P.Renderer(cfg)
    r.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    r.bind_image(image.data_ptr(), keepalive=image)
    r.allocateOnGPU(scene)
    # warmup: builds the primary-hit cache, warms caches/clocks; distinct iteration ids
    r.renderLoop(first_iter=iter_base + rank * max(W, 1), n_iters=W, sync=False)
    torch.cuda.synchronize(dev)
    if reduce_image and ctx.world > 1:
        # warm the accumulator-sized all-reduce: one-time RCCL setup is paid here
        ctx.dist.all_reduce(image, op=ctx.dist.ReduceOp.SUM)
        torch.cuda.synchronize(dev)
    r.clearImage()
    seg0 = r.segments()
    pb0 = r.segments_per_bounce()
    if events:
        r.kernel_stats()                   # reset
        r.set_profiling(2)                 # event pairs around pipeline 0's trace phases only
    ctx.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    r.renderLoop(first_iter=rank * K, n_iters=K, sync=False)
    if reduce_image and ctx.world > 1:
        ctx.dist.all_reduce(image, op=ctx.dist.ReduceOp.SUM)      # RCCL over xGMI
    torch.cuda.synchronize(dev)
    ctx.barrier()
    t1 = time.perf_counter()
    stats = r.kernel_stats() if events else None
    seg = r.segments() - seg0
    per_bounce = [a - b for a, b in zip(r.segments_per_bounce(), pb0)]
    while per_bounce and per_bounce[-1] == 0:
        per_bounce.pop()
    faults = r.trace_faults()
    img_ok = bool(torch.isfinite(image).all().item())
    pipes = r.pipelines()
    r.free()
    # every rank learns of a fault on any rank and stops together (no rank left in a collective)
    fmax, elapsed = ctx.reduce([float(faults), t1 - t0], "max")
    seg_total, seg0_total = ctx.reduce([float(seg), float(per_bounce[0] if per_bounce else 0)], "sum")
    if fmax > 0:
        raise SystemExit(f"bench: persistent-trace wave(s) hit the iteration cap on some rank "
                         f"(max {int(fmax)}); result invalid")
    return dict(elapsed=elapsed, seg=seg_total, seg_primary=seg0_total, per_bounce=per_bounce, stats=stats,
                img_ok=img_ok, pipes=pipes, faults=int(fmax))


def rates(res, K, npix, world):
    e = res["elapsed"]
    return {"value": round(res["seg"] / e / 1e6, 3), "unit": "Mrays/s",
            "traced_mrays_per_sec": round((res["seg"] - res["seg_primary"]) / e / 1e6, 3),
            "ms_per_step": round(e / K * 1e3, 3), "samples_per_sec": round(world * K * npix / e, 1)}


def trace_bytes_per_step(per_bounce, K):
    """Algorithmic HBM bytes of the persistent trace per step: every segment entering
    bounce b >= 1 reads its ray (o, d: 32 B) and writes its 20-B hit record."""
    return 52.0 * sum(per_bounce[1:]) / K


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
    ctx = Ctx(torch, dist, dev, rank, world)

    import pathtracerap_amd as P
    from pathtracerap_amd import synthetic

    accels = {"bvh": P.ACCEL_BVH, "grid": P.ACCEL_GRID, "grid_fast": P.ACCEL_GRID_FAST}
    tmp = tempfile.mkdtemp(prefix=f"ptbench_r{rank}_")
    if args.scene:
        scene_path = os.path.abspath(args.scene)
    else:
        scene_path = synthetic.diffuse_scene(tmp, ntri=args.ntri, width=args.width, height=args.height,
                                             bounces=args.bounces, accel=args.accel, metallic=args.metallic)
    accel = accels[args.accel]
    scene = P.Scene(scene_path)
    cfg = scene.apply_settings(P.RenderConfig())
    cfg.width, cfg.height, cfg.accel = args.width, args.height, accel
    if not args.scene:
        cfg.max_bounces = args.bounces
    args.bounces = cfg.max_bounces
    if args.pipelines > 0:
        cfg.pipelines = args.pipelines
    scene.build(grid=cfg.grid, bvh=accel != P.ACCEL_GRID)
    ntri = scene.counts()["nt"]
    npix = cfg.width * cfg.height
    K, W = args.steps, args.warmup
    events = not args.no_profile

    main_res = timed_run(P, ctx, scene, cfg, K, W, 1_000_000, events, reduce_image=True)
    per_bounce = main_res["per_bounce"]
    workload_key = f"{args.accel}_{args.ntri}_{args.width}x{args.height}_b{args.bounces}" + \
        ("_metal" if args.metallic else "")

    # Per-kernel durations of ONE pipeline, for comparison with the timed run's
    # overlapping launches: a separate pass of the same K iterations (same ids =>
    # the same per-bounce ray counts), rank 0 only while the others wait.
    stats1 = None
    if events and rank == 0:
        cfg_p = P.RenderConfig(**{**cfg.__dict__, "pipelines": 1})
        image = torch.zeros(npix * 3, dtype=torch.float32, device=dev)
        rp = P.Renderer(cfg_p)
        rp.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        rp.bind_image(image.data_ptr(), keepalive=image)
        rp.allocateOnGPU(scene)
        rp.renderLoop(first_iter=1_000_000, n_iters=W, sync=False)
        torch.cuda.synchronize(dev)
        rp.kernel_stats()          # reset
        rp.set_profiling(True)
        rp.renderLoop(first_iter=rank * K, n_iters=K, sync=True)
        stats1 = rp.kernel_stats()
        rp.free()
    ctx.barrier()

    alt = None
    if args.alt_accel and args.alt_accel != args.accel:
        acc2 = accels[args.alt_accel]
        cfg2 = P.RenderConfig(**{**cfg.__dict__, "accel": acc2})
        if acc2 != P.ACCEL_GRID and accel == P.ACCEL_GRID:
            scene.build(grid=cfg.grid, bvh=True)
        ra = timed_run(P, ctx, scene, cfg2, K, W, 2_000_000, False, reduce_image=False)
        alt = {"accel": args.alt_accel, **rates(ra, K, npix, world),
               "semantics": "exact closest hit (statistically equivalent image, not per-pixel identical)"
               if args.alt_accel == "bvh" else "reference grid (bit-identical)"}

    targets = {}
    tk = max(1, min(K, args.target_steps))
    for name in [t for t in args.targets.split(",") if t]:
        if name == "target_1m":
            path = synthetic.diffuse_scene(tmp, ntri=1_000_000, accel=args.accel)
            st = P.Scene(path)
            ct = st.apply_settings(P.RenderConfig())
            label = ("north_star target: 1M-triangle diffuse synthetic OBJ, 1280x1024, 8 bounces "
                     "(north_star asks 1024 spp: per-step rate)")
        elif name == "configs2":
            st = P.Scene(os.path.join(ROOT, "scenes", "reference_scene.txt"))
            ct = st.apply_settings(P.RenderConfig())
            ct.width, ct.height = 2800, 2240
            label = ("configs[2]: the README render's scene (Scene.cpp:3-224: metal, coat, diffuse, emissive "
                     "models), 2800x2240, the reference's 5 bounces (configs[2] asks 1024 spp: per-step rate)")
        else:
            raise SystemExit(f"bench: unknown target {name}")
        ct.accel = accel
        if args.pipelines > 0:
            ct.pipelines = args.pipelines
        st.build(grid=ct.grid, bvh=accel != P.ACCEL_GRID)
        rt = timed_run(P, ctx, st, ct, tk, min(W, 2), 3_000_000, False, reduce_image=True)
        targets[name] = {"workload": label, "triangles": st.counts()["nt"], "width": ct.width,
                         "height": ct.height, "bounces": ct.max_bounces, "steps": tk, **rates(rt, tk, ct.width * ct.height, world),
                         "segments": int(rt["seg"]), "image_finite": rt["img_ok"], "trace_faults": rt["faults"]}
        del st

    if rank == 0:
        r_main = rates(main_res, K, npix, world)
        roof = None
        stats = main_res["stats"]
        if stats and stats.get("trace_launches", 0) > 0:
            # Dominant kernel: the persistent trace of bounces >= 1 (k_trace_gf / k_trace_bvh).
            # Algorithmic bytes per segment entering bounce b >= 1: 32 B ray read (o, d) + 20 B
            # hit record write.  `achieved` = those bytes per step / ms_per_step: the launches of
            # the 16 iterations in flight overlap, so the step's wall time is the time the
            # kernel's work takes (a slight under-estimate: the other kernels share that time).
            kname = "k_trace_bvh" if args.accel == "bvh" else "k_trace_gf"
            tb_step = trace_bytes_per_step(per_bounce, K)
            phases = max(1, len(per_bounce) - 1)                 # trace phases per step
            job = tb_step / (main_res["elapsed"] / K) / 1e9      # per GPU: each rank runs K steps
            # one "launch" = one bounce's trace phase (main launch + tail launches +
            # k_trace_deferred), timed by an event pair on pipeline 0's stream in the timed region
            launches = stats["trace_launches"]
            kms = stats["trace_ms"] / launches
            b_launch = tb_step / phases
            a_launch = b_launch / (kms / 1e3) / 1e9
            tr = load_pmc(kname, workload_key)                   # HBM bytes per launch, one pipeline
            roof = {"bound": "hbm", "achieved": round(job, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(job / HBM_PEAK_GBS, 5),
                    "traffic": None if tr is None else round(tr * phases),
                    "kernel": kname, "basis": "per step: algorithmic trace bytes per step / ms_per_step "
                                              "(traffic: PMC HBM bytes per launch x trace phases per step)",
                    "algorithmic_bytes_per_step": round(tb_step), "ms_per_step": r_main["ms_per_step"],
                    "trace_phases_per_step": phases, "traffic_per_launch": None if tr is None else round(tr),
                    "per_launch": {
                        "avg_launch_ms": round(kms, 4), "algorithmic_bytes_per_launch": round(b_launch),
                        "achieved": round(a_launch, 2), "frac": round(a_launch / HBM_PEAK_GBS, 5),
                        "launches_timed": launches, "pipelines": main_res["pipes"],
                        "measured": "HIP event pair around each of pipeline 0's trace phases inside the timed "
                                    "region: from the phase's turn on its stream to its last launch's end, so it "
                                    "includes waiting for CU slots the other pipelines' kernels hold (rocprofv3 "
                                    "times execution only: profiles/r03/kernel_stats_grid_fast_16p.csv)",
                        "why_launches_exceed_step": (
                            f"{phases} trace phases per step x {kms:.3f} ms = {phases * kms:.2f} ms of launch "
                            f"time per step against {r_main['ms_per_step']:.3f} ms per step: "
                            f"{main_res['pipes']} iterations are in flight, so about "
                            f"{phases * kms / r_main['ms_per_step']:.1f} trace phases run at once")}}
            if stats1 and stats1.get("trace_launches", 0) > 0:
                l1 = stats1["trace_launches"]
                k1 = stats1["trace_ms"] / l1
                a1 = b_launch / (k1 / 1e3) / 1e9
                roof["single_pipeline"] = {"avg_launch_ms": round(k1, 4), "achieved": round(a1, 2),
                                           "frac": round(a1 / HBM_PEAK_GBS, 5), "launches": l1,
                                           "sort_avg_ms": round(stats1["sort_ms"] / max(stats1["sort_launches"], 1), 4),
                                           "shade_avg_ms": round(stats1["bounce_ms"] / max(stats1["bounce_launches"], 1), 4),
                                           "scan_avg_ms": round(stats1["scan_ms"] / max(stats1["scan_launches"], 1), 4),
                                           "measured": "HIP events, a separate pass of the same iterations with one "
                                                       "pipeline (no overlap), rank 0"}
        # Issue roofline: the traces are bound by instruction issue and dependent-load
        # latency, not by HBM bytes, so the VALU issue rate against the SIMDs' peak is
        # the informative fraction -- for the whole job (all kernels of a step, with the
        # pipelines overlapping) and for the dominant kernel's single-pipeline launches.
        issue = None
        sq = load_sq(workload_key)
        if sq:
            v_step = sq["valu_insts_per_iteration"]
            job = v_step * K / main_res["elapsed"] / 1e9      # per GPU: each rank runs K steps in `elapsed`
            issue = {"bound": "valu", "unit": "G wave-instr/s", "peak": VALU_PEAK_G,
                     "job": {"valu_insts_per_step": round(v_step), "achieved": round(job, 1),
                             "frac": round(job / VALU_PEAK_G, 4),
                             "salu_insts_per_step": round(sq["salu_insts_per_iteration"]),
                             "salu_achieved": round(sq["salu_insts_per_iteration"] * K / main_res["elapsed"] / 1e9, 1)},
                     "source": "rocprofv3 SQ_INSTS_VALU / SQ_INSTS_SALU pass (profiles/pmc_latest.json)"}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(scene_path, args.bounces, cfg.width, cfg.height, args.cpu_seconds)
            except Exception as e:  # noqa: BLE001 -- reported, not fatal
                cpu = {"error": repr(e)}
        out = {
            "metric": METRIC, "value": r_main["value"], "unit": "Mrays/s", "n_gpus": world, "steps": K,
            "warmup": W, "ms_per_step": r_main["ms_per_step"], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "samples_per_sec": r_main["samples_per_sec"],
            "traced_mrays_per_sec": r_main["traced_mrays_per_sec"],
            "config": {"workload": workload_name(args),
                       "triangles": ntri, "width": cfg.width, "height": cfg.height, "bounces": cfg.max_bounces,
                       "spp_per_step": 1, "accel": args.accel,
                       "results": "bit-identical to the reference algorithm (oracle-checked at this size: "
                                  "tests/test_gpu_configs.py)" if args.accel != "bvh" else "exact closest hit",
                       "parallelism": f"samples sharded x{world}" + (" (gloo rehearsal)" if world > 1 and args.dist_backend == "gloo" else ""),
                       "pipelines": main_res["pipes"],
                       "segments": int(main_res["seg"]), "primary_segments_cached": int(main_res["seg_primary"]),
                       "segments_per_bounce_rank0": per_bounce,
                       "image_finite": main_res["img_ok"], "trace_faults": main_res["faults"]},
            "roofline": roof, "issue_roofline": issue, "cpu_baseline": cpu, "alt_mode": alt,
            "targets": targets or None,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
