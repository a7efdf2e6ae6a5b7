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
resident in HBM before the timed region starts.  ``targets`` times more
workloads the same way: north_star's target (the 1M-triangle diffuse OBJ at
1280x1024), configs[2] (the README render's own scene, Scene.cpp:3-224, at
2800x2240) and configs[4] (the 10M-triangle scene, 16 bounces).  Each
workload also renders its configuration's own sample count once (``full_run``:
256 spp for configs[1], 1024 for the target and configs[2], 4096 for
configs[4]; the reference's ITER, Config.h:19), timed the same way.

Multi-GPU: ``--gpus N`` with N > 1 starts N ranks itself (one process per GPU,
MASTER_ADDR 127.0.0.1) unless a launcher already set WORLD_SIZE
(``torchrun --nproc-per-node N bench.py --gpus N``); either way the world size
must equal N.  Samples shard across ranks (rank r renders iterations
[r*K, (r+1)*K)), then one RCCL all-reduce sums the float3 accumulator; weak
scaling.

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
import signal
import socket
import subprocess
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
# samples per pixel each BASELINE.json configuration asks for (full_run)
SPP = {"configs1": 256, "target_1m": 1024, "configs2": 1024, "configs4": 4096}
# What "bit-exact" means here: the reference is CUDA + thrust + Assimp + MSVC and
# cannot be built in this image, so parity is against its C restatement, which is
# pinned to the reference's own output image (tests/golden/oracle_pin_stats.json)
PARITY_BASIS = ("bit-exact vs the C restatement of the reference algorithm (oracle/ptoracle.c; checked at this "
                "size by tests/test_gpu_configs.py); the restatement is within 1 LSB of the reference's Render.bmp "
                "on 99.4 % of channels (max 4), not bit-exact vs the CUDA binary, which cannot be built here")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=0,
                    help="GPUs (ranks); 0: WORLD_SIZE when a launcher set it, else 1.  N > 1 without a launcher: "
                         "bench.py starts the N ranks itself")
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
    ap.add_argument("--inmem", action="store_true", help="build the synthetic scene in memory (addMesh / addModel) "
                                                        "instead of through OBJ text (10M triangles: minutes of text)")
    ap.add_argument("--scene", default="", help="a scene file instead of the synthetic OBJ scene (e.g. "
                                                "scenes/reference_scene.txt); its RENDER block's bounces apply")
    ap.add_argument("--targets", default="target_1m,configs2,configs4",
                    help="extra workloads timed after the main line ('' to skip): target_1m = north_star's "
                         "1M-triangle scene at 1280x1024; configs2 = the README scene at 2800x2240; configs4 = "
                         "the 10M-triangle scene at 1280x1024, 16 bounces")
    ap.add_argument("--target-steps", type=int, default=16)
    ap.add_argument("--no-full-runs", action="store_true",
                    help="skip the full-spp renders (256 / 1024 / 1024 / 4096 spp) of each workload")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU baseline duration")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="no one-pipeline HIP-event pass (roofline)")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="process group for N>1 (nccl = RCCL over xGMI; gloo only to rehearse the "
                         "multi-rank path with several ranks on one GPU)")
    ap.add_argument("--pipelines", type=int, default=16,
                    help="iterations in flight on their own HIP streams (0: the library default, 16)")
    ap.add_argument("--hw-queues", type=int, default=16,
                    help="GPU_MAX_HW_QUEUES for this process (HIP default 4): one hardware queue per "
                         "pipeline stream (max 32)")
    return ap.parse_args(argv)


def spawn_ranks(n, argv):
    """--gpus N without a launcher: start ranks 0..N-1 of this script as child
    processes (nothing here has touched the GPU: the parent only waits), rank 0's
    stdout is the JSON line.  If a rank fails, the others are stopped (they would
    wait in a collective forever) and the failing exit code is returned."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      start_new_session=True))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                print(f"bench: rank {procs.index(p)} exited with {code}; stopping the other ranks", file=sys.stderr)
                for q in live:
                    try:
                        os.killpg(q.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
                deadline = time.time() + 15
                for q in live:
                    try:
                        q.wait(timeout=max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        try:
                            os.killpg(q.pid, signal.SIGKILL)
                        except ProcessLookupError:
                            pass
                        q.wait()
                live = []
                break
        time.sleep(0.1)
    return rc


def host_cpu_share():
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU quota
    and by the pool's per-GPU share (OMP_NUM_THREADS, set on the GPU box) when
    those exist.  Returns (threads, description)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    n, why = aff, [f"affinity mask {aff} CPUs"]
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            q = max(1, int(int(quota) / int(period)))
            why.append(f"cgroup quota {q} CPUs")
            n = min(n, q)
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        why.append(f"OMP_NUM_THREADS {omp} (the pool's CPU share per GPU)")
        n = min(n, int(omp))
    return max(1, n), ", ".join(why)


def cpu_baseline(scene, bounces, width, height, target_s):
    """The oracle (C port of the reference's bounce loop) on the host cores:
    same scene (the built product Scene's export) and camera, reduced
    resolution, 1 sample per pixel, sized to about ``target_s`` seconds of CPU
    work."""
    import oracle as O
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import flat_from_export

    threads, share = host_cpu_share()
    flat = flat_from_export(scene.export())

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
    return {"value": seg / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port", "cpu_share": share,
            "sample": f"oracle/ptoracle.c (C port of the reference renderLoop, uniform-grid accel as in "
                      f"the reference, OpenMP over rays) on the same scene/camera at {w}x{h}, {iters} spp, "
                      f"{bounces} bounces: {seg} segments in {dt:.2f}s on {threads} thread(s) ({share})"}


def workload_name(args):
    """Label of the BASELINE.json configuration this run measures."""
    if args.scene:
        return f"scene file {os.path.relpath(args.scene, ROOT)}, {args.width}x{args.height}, {args.bounces} bounces"
    if is_default_workload(args):
        return "configs[1]: diffuse-only synthetic OBJ (~100k tris), 1280x1024, 8 bounces"
    kind = "metallic+diffuse" if args.metallic else "diffuse-only"
    tag = ""
    if not args.metallic and args.ntri >= 5_000_000:
        tag = "configs[4] shape: "
    elif not args.metallic and args.ntri >= 500_000:
        tag = "north_star target shape: "
    return f"{tag}{kind} synthetic OBJ (~{args.ntri} tris), {args.width}x{args.height}, {args.bounces} bounces"


def is_default_workload(args):
    return (not args.scene and args.ntri == 100_000 and args.width == 1280 and args.height == 1024
            and args.bounces == 8 and not args.metallic)


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
    """Process-group plumbing shared by every timed workload.  ``pg``: a process
    group exists (a launcher or bench.py's own spawner set WORLD_SIZE, also at
    world size 1), so the accumulator all-reduce and the max-over-ranks run through
    it exactly as on N GPUs."""

    def __init__(self, torch, dist, dev, rank, world, pg=False):
        self.torch, self.dist, self.dev, self.rank, self.world, self.pg = torch, dist, dev, rank, world, pg

    def barrier(self):
        if self.pg:
            self.dist.barrier()

    def reduce(self, vals, op):
        """vals (floats) reduced over ranks with op ('max' / 'sum')."""
        t = self.torch.tensor(vals, dtype=self.torch.float64, device=self.dev)
        if self.pg:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM)
        return [float(x) for x in t.cpu()]


def check_backend(backend, world, ngpu):
    """RCCL needs one GPU per rank: more ranks than visible GPUs would map two
    ranks onto one device, and init_process_group then fails or hangs.  Checked
    before any process-group or GPU call; returns an error string or None."""
    if backend == "nccl" and world > ngpu:
        return (f"bench: --dist-backend nccl with {world} rank(s) but {ngpu} visible GPU(s); RCCL needs one "
                f"GPU per rank (use --dist-backend gloo to rehearse several ranks on one GPU)")
    return None


def bound_fracs(obj, path="line"):
    """Every ``frac`` in the line is a fraction of a hardware peak: one above 1
    (or not finite) is a measurement error, so it is published as null beside an
    ``error`` key instead of as a number.  Returns the paths it nulled."""
    bad = []
    if isinstance(obj, dict):
        for k, v in list(obj.items()):
            if k == "frac" and v is not None:
                if not (isinstance(v, (int, float)) and 0.0 <= v <= 1.0):
                    obj["frac"] = None
                    obj["error"] = f"frac {v!r} outside [0, 1]: inconsistent counters, not published"
                    bad.append(path)
            else:
                bad += bound_fracs(v, f"{path}.{k}")
    elif isinstance(obj, list):
        for i, v in enumerate(obj):
            bad += bound_fracs(v, f"{path}[{i}]")
    return bad


def timed_run(P, ctx, scene, cfg, K, W, iter_base, reduce_image, full_spp=0):
    """Warm up, then time exactly K iterations (this rank's [rank*K, (rank+1)*K))
    between barrier + synchronize pairs; the accumulator all-reduce (RCCL) is
    inside the timed region.  No profiling events in the timed region.  With
    ``full_spp`` the same renderer then renders iterations [0, full_spp) sharded
    over the ranks (the configuration's own sample count), timed the same way.
    Trace faults (waves that hit the iteration cap) of the warmup and of both
    timed regions make the run invalid.  Returns the max-over-ranks times, the
    all-rank segment totals and the per-bounce counts of rank 0's K steps."""
    from pathtracerap_amd.dist import shard_iterations
    torch, dev, rank, world = ctx.torch, ctx.dev, ctx.rank, ctx.world
    image = torch.zeros(cfg.width * cfg.height * 3, dtype=torch.float32, device=dev)
    r = P.Renderer(cfg)
    r.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    r.bind_image(image.data_ptr(), keepalive=image)
    r.allocateOnGPU(scene)
    # warmup: builds the primary-hit cache, warms caches/clocks; distinct iteration ids
    r.renderLoop(first_iter=iter_base + rank * max(W, 1), n_iters=W, sync=False)
    torch.cuda.synchronize(dev)
    faults = r.trace_faults()          # clearImage resets the counter: read the warmup's first
    if reduce_image and ctx.pg:
        # warm the accumulator-sized all-reduce: one-time RCCL setup is paid here
        ctx.dist.all_reduce(image, op=ctx.dist.ReduceOp.SUM)
        torch.cuda.synchronize(dev)

    def region(first, n):
        r.clearImage()
        ctx.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        r.renderLoop(first_iter=first, n_iters=n, sync=False)
        if reduce_image and ctx.pg:
            ctx.dist.all_reduce(image, op=ctx.dist.ReduceOp.SUM)      # RCCL over xGMI
        torch.cuda.synchronize(dev)
        ctx.barrier()
        return time.perf_counter() - t0

    seg0, pb0 = r.segments(), r.segments_per_bounce()
    elapsed = region(rank * K, K)
    faults += r.trace_faults()
    seg = r.segments() - seg0
    per_bounce = [a - b for a, b in zip(r.segments_per_bounce(), pb0)]
    while per_bounce and per_bounce[-1] == 0:
        per_bounce.pop()
    img_ok = bool(torch.isfinite(image).all().item())
    full = None
    if full_spp > 0:
        first, n = shard_iterations(full_spp, rank, world)
        segf0, pbf0 = r.segments(), r.segments_per_bounce(1)[0]
        el_full = region(first, n)
        faults += r.trace_faults()
        full = [el_full, float(r.segments() - segf0), float(r.segments_per_bounce(1)[0] - pbf0),
                float(torch.isfinite(image).all().item())]
    pipes = r.pipelines()
    r.free()
    # every rank learns of a fault on any rank and stops together (no rank left in a collective)
    fmax, el_max = ctx.reduce([float(faults), elapsed], "max")
    seg_total, seg0_total = ctx.reduce([float(seg), float(per_bounce[0] if per_bounce else 0)], "sum")
    if fmax > 0:
        raise SystemExit(f"bench: persistent-trace wave(s) hit the iteration cap on some rank "
                         f"(max {int(fmax)}); result invalid")
    res = dict(elapsed=el_max, seg=seg_total, seg_primary=seg0_total, per_bounce=per_bounce, img_ok=img_ok,
               pipes=pipes, faults=int(fmax))
    if full is not None:
        fel, = ctx.reduce([full[0]], "max")
        fseg, fseg0, fok = ctx.reduce(full[1:], "sum")
        res["full"] = dict(spp=full_spp, elapsed=fel, seg=fseg, seg_primary=fseg0, img_ok=fok == world)
    return res


def rates(res, K, npix, world):
    e = res["elapsed"]
    return {"value": round(res["seg"] / e / 1e6, 3), "unit": "Mrays/s",
            "traced_mrays_per_sec": round((res["seg"] - res["seg_primary"]) / e / 1e6, 3),
            "ms_per_step": round(e / K * 1e3, 3), "samples_per_sec": round(world * K * npix / e, 1)}


def full_rates(res, npix):
    """The full-spp render: spp iterations over all ranks in `elapsed` seconds."""
    f = res.get("full")
    if not f:
        return None
    e = f["elapsed"]
    return {"spp": f["spp"], "seconds": round(e, 4), "value": round(f["seg"] / e / 1e6, 3), "unit": "Mrays/s",
            "traced_mrays_per_sec": round((f["seg"] - f["seg_primary"]) / e / 1e6, 3),
            "samples_per_sec": round(f["spp"] * npix / e, 1), "segments": int(f["seg"]), "image_finite": f["img_ok"]}


def trace_bytes_per_step(per_bounce, K):
    """Algorithmic HBM bytes of the persistent trace per step: every segment entering
    bounce b >= 1 reads its ray (o, d: 32 B) and writes its 20-B hit record."""
    return 52.0 * sum(per_bounce[1:]) / K


def one_pipeline_pass(P, torch, dev, scene, cfg, K, W):
    """Per-kernel HIP-event durations of ONE pipeline (no overlapping launches):
    the same K iterations as the timed region (same ids => the same per-bounce
    ray counts), events recorded on the pipeline's stream around every kernel
    group (renderer profiling level 1)."""
    cfg_p = P.RenderConfig(**{**cfg.__dict__, "pipelines": 1})
    image = torch.zeros(cfg.width * cfg.height * 3, dtype=torch.float32, device=dev)
    rp = P.Renderer(cfg_p)
    rp.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    rp.bind_image(image.data_ptr(), keepalive=image)
    rp.allocateOnGPU(scene)
    rp.set_profiling(1)        # the warmup's first renderLoop builds the primary-hit cache (k_primary): timed
    rp.renderLoop(first_iter=1_000_000, n_iters=W, sync=False)
    torch.cuda.synchronize(dev)
    primary_ms = rp.kernel_stats()["primary_ms"]     # reads and resets
    rp.renderLoop(first_iter=0, n_iters=K, sync=True)
    st = rp.kernel_stats()
    st["primary_ms"] = primary_ms
    rp.free()
    return st


def target_key(accel, name, cfg):
    """pmc_latest.json key of a target workload: the key its own main-line run
    (bench.py --ntri N --bounces B [--inmem]) writes, so scripts/round_profiles.sh's
    per-target counter passes line up with the targets' one-pipeline passes."""
    ntri = {"target_1m": 1_000_000, "configs4": 10_000_000}.get(name)
    if ntri is None:
        return f"{accel}_{name}_{cfg.width}x{cfg.height}_b{cfg.max_bounces}"
    return f"{accel}_{ntri}_{cfg.width}x{cfg.height}_b{cfg.max_bounces}"


def trace_roofline(stats1, per_bounce, K, elapsed, ms_per_step, kname, workload_key):
    """Roofline of the dominant kernel, the persistent trace of bounces >= 1
    (k_trace_gf / k_trace_bvh), per launch.  Algorithmic bytes per segment
    entering bounce b >= 1: 32 B ray read (o, d) + 20 B hit record write; one
    "launch" = one bounce's trace phase, timed by a HIP event pair on the stream
    it is launched on, with one pipeline (no overlap, no drain tail).  Beside it:
    the PMC HBM bytes of the same launches (traffic), their VALU issue rate and
    the wave-cycle split, all from profiles/pmc_latest.json under workload_key."""
    if not stats1 or stats1.get("trace_launches", 0) <= 0:
        return None
    tb_step = trace_bytes_per_step(per_bounce, K)
    phases = max(1, len(per_bounce) - 1)                 # trace phases per step
    b_launch = tb_step / phases                          # algorithmic bytes per launch (one bounce's trace)
    job = tb_step / (elapsed / K) / 1e9                  # per GPU: each rank runs K steps
    l1 = stats1["trace_launches"]
    k1 = stats1["trace_ms"] / l1
    a1 = b_launch / (k1 / 1e3) / 1e9
    tr = load_pmc(kname, workload_key)                   # PMC HBM bytes per launch, one pipeline
    roof = {"bound": "hbm", "achieved": round(a1, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(a1 / HBM_PEAK_GBS, 5), "traffic": None if tr is None else round(tr),
            "kernel": kname, "workload_key": workload_key,
            "basis": "per launch: algorithmic bytes of one bounce's trace (52 B x segments entering the bounce) "
                     "/ its average duration, HIP events on the launch stream, one pipeline (rocprofv3: "
                     "profiles/r06/kernel_stats_*_1p.csv); traffic = PMC HBM bytes per launch of the same "
                     "command, (2 FETCH_SIZE + WRITE_SIZE) KiB (profiles/pmc_latest.json)",
            "algorithmic_bytes_per_launch": round(b_launch), "avg_launch_ms": round(k1, 4),
            "launches": l1, "trace_phases_per_step": phases,
            "per_step": {"achieved": round(job, 2), "frac": round(job / HBM_PEAK_GBS, 5),
                         "algorithmic_bytes_per_step": round(tb_step), "ms_per_step": ms_per_step,
                         "note": "whole-job rate: algorithmic trace bytes per step / ms_per_step (the iterations "
                                 "in flight share the step's wall time)"},
            "sort_avg_ms": round(stats1["sort_ms"] / max(stats1["sort_launches"], 1), 4),
            "primary_cache_ms": round(stats1.get("primary_ms", 0.0), 4),   # k_primary, once per renderer
            "shade_avg_ms": round(stats1["bounce_ms"] / max(stats1["bounce_launches"], 1), 4),
            "scan_avg_ms": round(stats1["scan_ms"] / max(stats1["scan_launches"], 1), 4)}
    if tr is not None:
        roof["traffic_over_algorithmic"] = round(tr / max(b_launch, 1.0), 2)
    sq1 = load_sq(workload_key, "_sq_p1")
    kv = (sq1 or {}).get("kernels", {}).get(kname)
    if kv:
        g = kv["valu_insts_per_launch"] / (k1 / 1e3) / 1e9
        roof["issue"] = {"bound": "valu", "unit": "G wave-instr/s", "peak": VALU_PEAK_G,
                         "valu_insts_per_launch": round(kv["valu_insts_per_launch"]),
                         "achieved": round(g, 1), "frac": round(g / VALU_PEAK_G, 4),
                         "source": "rocprofv3 SQ_INSTS_VALU pass, one pipeline (profiles/pmc_latest.json) "
                                   "/ avg_launch_ms"}
    cyc = (load_sq(workload_key, "_cycles_p1") or {}).get(f"{kname}.main")
    if cyc:
        roof["wave_cycles"] = {k: round(cyc[k], 4) for k in ("wait_share", "issue_stall_share", "active_share",
                                                              "lanes_per_valu") if k in cyc}
        roof["wave_cycles"]["source"] = "rocprofv3 SQ wave-cycle pass, one pipeline (profiles/pmc_latest.json)"
    return roof


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # no launcher: start the ranks here, before anything touches the GPU
        if args.hw_queues > 0:
            os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, args.hw_queues))
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    if args.gpus and args.gpus != world:
        raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started {world} rank(s)")
    if args.hw_queues > 0:     # read once by the HIP runtime at initialisation: set before torch touches it
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, args.hw_queues))
    # torch first: its HIP runtime is the process's (libpathtracer_amd.so then binds to it; loaded
    # before torch, the library's own /opt/rocm runtime left torch's allocations without a device)
    import torch
    import torch.distributed as dist

    import pathtracerap_amd as P

    # one rank per GPU (RCCL); only a gloo rehearsal may put several ranks on one
    # GPU (round-robin).  device_count() does not initialise HIP on this image.
    ngpu = torch.cuda.device_count()
    pg = env_world is not None                # a launcher (or spawn_ranks): a process group, even at world 1
    if pg:
        err = check_backend(args.dist_backend, world, ngpu)
        if err:
            raise SystemExit(err)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, ngpu)
    if pg:
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    ctx = Ctx(torch, dist, dev, rank, world, pg)

    from pathtracerap_amd import synthetic

    accels = {"bvh": P.ACCEL_BVH, "grid": P.ACCEL_GRID, "grid_fast": P.ACCEL_GRID_FAST}
    tmp = tempfile.mkdtemp(prefix=f"ptbench_r{rank}_")
    accel = accels[args.accel]
    if args.inmem and not args.scene:
        scene = synthetic.build_scene(P, args.ntri, metallic=args.metallic, bvh=accel != P.ACCEL_GRID)
        cfg = P.RenderConfig()
    else:
        if args.scene:
            scene_path = os.path.abspath(args.scene)
        else:
            scene_path = synthetic.diffuse_scene(tmp, ntri=args.ntri, width=args.width, height=args.height,
                                                 bounces=args.bounces, accel=args.accel, metallic=args.metallic)
        scene = P.Scene(scene_path)
        cfg = scene.apply_settings(P.RenderConfig())
    cfg.width, cfg.height, cfg.accel = args.width, args.height, accel
    if not args.scene:
        cfg.max_bounces = args.bounces
    args.bounces = cfg.max_bounces
    if args.pipelines > 0:
        cfg.pipelines = args.pipelines
    if not (args.inmem and not args.scene):
        scene.build(grid=cfg.grid, bvh=accel != P.ACCEL_GRID)
    ntri = scene.counts()["nt"]
    npix = cfg.width * cfg.height
    K, W = args.steps, args.warmup
    full_main = 0 if args.no_full_runs or not is_default_workload(args) else SPP["configs1"]

    main_res = timed_run(P, ctx, scene, cfg, K, W, 1_000_000, reduce_image=True, full_spp=full_main)
    per_bounce = main_res["per_bounce"]
    workload_key = f"{args.accel}_{args.ntri}_{args.width}x{args.height}_b{args.bounces}" + \
        ("_metal" if args.metallic else "")

    # Per-kernel durations of ONE pipeline (rank 0 while the others wait): the
    # dominant kernel's launches without the overlap of the 16 iterations in flight
    stats1 = None
    if not args.no_profile and rank == 0:
        stats1 = one_pipeline_pass(P, torch, dev, scene, cfg, K, W)
    ctx.barrier()

    alt = None
    if args.alt_accel and args.alt_accel != args.accel:
        acc2 = accels[args.alt_accel]
        cfg2 = P.RenderConfig(**{**cfg.__dict__, "accel": acc2})
        if acc2 != P.ACCEL_GRID and accel == P.ACCEL_GRID:
            scene.build(grid=cfg.grid, bvh=True)
        ra = timed_run(P, ctx, scene, cfg2, K, W, 2_000_000, reduce_image=False)
        alt = {"accel": args.alt_accel, **rates(ra, K, npix, world),
               "semantics": "exact closest hit (statistically equivalent image, not per-pixel identical)"
               if args.alt_accel == "bvh" else "reference grid (bit-identical)"}

    targets = {}
    tk = max(1, min(K, args.target_steps))
    for name in [t for t in args.targets.split(",") if t]:
        t_build = time.perf_counter()
        if name == "target_1m":
            path = synthetic.diffuse_scene(tmp, ntri=1_000_000, accel=args.accel)
            st = P.Scene(path)
            ct = st.apply_settings(P.RenderConfig())
            label = "north_star target: 1M-triangle diffuse synthetic OBJ, 1280x1024, 8 bounces"
        elif name == "configs2":
            st = P.Scene(os.path.join(ROOT, "scenes", "reference_scene.txt"))
            ct = st.apply_settings(P.RenderConfig())
            ct.width, ct.height = 2800, 2240
            label = ("configs[2]: the README render's scene (Scene.cpp:3-224: metal, coat, diffuse, emissive "
                     "models), 2800x2240, the reference's 5 bounces")
        elif name == "configs4":
            # built in memory (addMesh / addModel): the 10M-triangle OBJ text would take
            # about a minute to write and parse; same layout as diffuse_scene
            st = None
            ct = P.RenderConfig(width=1280, height=1024, max_bounces=16)
            label = ("configs[4]: synthetic 10M-triangle diffuse scene (displaced torus in the room, deep BLAS), "
                     "1280x1024, 16 bounces")
        else:
            raise SystemExit(f"bench: unknown target {name}")
        ct.accel = accel
        if args.pipelines > 0:
            ct.pipelines = args.pipelines
        if st is None:
            st = synthetic.build_scene(P, 10_000_000, grid=ct.grid, bvh=accel != P.ACCEL_GRID)
        else:
            st.build(grid=ct.grid, bvh=accel != P.ACCEL_GRID)
        t_build = time.perf_counter() - t_build
        spp = 0 if args.no_full_runs else SPP[name]
        rt = timed_run(P, ctx, st, ct, tk, min(W, 2), 3_000_000, reduce_image=True, full_spp=spp)
        tnpix = ct.width * ct.height
        troof = None
        if not args.no_profile and rank == 0 and args.accel != "grid":
            tkey = target_key(args.accel, name, ct)
            st1 = one_pipeline_pass(P, torch, dev, st, ct, tk, min(W, 2))
            troof = trace_roofline(st1, rt["per_bounce"], tk, rt["elapsed"], round(rt["elapsed"] / tk * 1e3, 3),
                                   "k_trace_bvh" if args.accel == "bvh" else "k_trace_gf", tkey)
        ctx.barrier()
        targets[name] = {"workload": label, "triangles": st.counts()["nt"], "width": ct.width,
                         "height": ct.height, "bounces": ct.max_bounces, "steps": tk,
                         **rates(rt, tk, tnpix, world), "segments": int(rt["seg"]), "image_finite": rt["img_ok"],
                         "trace_faults": rt["faults"], "host_scene_build_s": round(t_build, 2),
                         "full_run": full_rates(rt, tnpix), "roofline": troof}
        del st

    if rank == 0:
        r_main = rates(main_res, K, npix, world)
        kname = "k_trace_bvh" if args.accel == "bvh" else "k_trace_gf"
        roof = None
        if args.accel != "grid":
            roof = trace_roofline(stats1, per_bounce, K, main_res["elapsed"], r_main["ms_per_step"], kname,
                                  workload_key)
        # Issue roofline of the whole job: the traces are bound by instruction issue and
        # dependent-load latency, not by HBM bytes, so the VALU issue rate (all kernels of
        # a step, the pipelines overlapping) against the SIMDs' peak is reported beside it.
        issue = None
        sq = load_sq(workload_key)
        if sq:
            v_step = sq["valu_insts_per_iteration"]
            g = v_step * K / main_res["elapsed"] / 1e9      # per GPU: each rank runs K steps in `elapsed`
            issue = {"bound": "valu", "unit": "G wave-instr/s", "peak": VALU_PEAK_G,
                     "job": {"valu_insts_per_step": round(v_step), "achieved": round(g, 1),
                             "frac": round(g / VALU_PEAK_G, 4),
                             "salu_insts_per_step": round(sq["salu_insts_per_iteration"]),
                             "salu_achieved": round(sq["salu_insts_per_iteration"] * K / main_res["elapsed"] / 1e9, 1)},
                     "iterations_counted": sq.get("iterations"),
                     "source": "rocprofv3 SQ_INSTS_VALU / SQ_INSTS_SALU pass at the bench's pipelines "
                               "(profiles/pmc_latest.json); per step = counts / first-bounce dispatches counted"}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(scene, args.bounces, cfg.width, cfg.height, args.cpu_seconds)
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
                       "results": PARITY_BASIS if args.accel != "bvh" else "exact closest hit",
                       "parallelism": f"samples sharded x{world}" + (
                           "" if not pg else " (gloo rehearsal)" if args.dist_backend == "gloo"
                           else " (RCCL all-reduce of the float3 accumulator)"),
                       "pipelines": main_res["pipes"], "hw_queues": P.hw_queues(),
                       "segments": int(main_res["seg"]), "primary_segments_cached": int(main_res["seg_primary"]),
                       "segments_per_bounce_rank0": per_bounce,
                       "image_finite": main_res["img_ok"], "trace_faults": main_res["faults"]},
            "full_run": full_rates(main_res, npix),
            "roofline": roof, "issue_roofline": issue, "cpu_baseline": cpu, "alt_mode": alt,
            "targets": targets or None,
        }
        nulled = bound_fracs(out)
        if nulled:
            print(f"bench: fraction(s) above 1 not published: {nulled}", file=sys.stderr)
        print(json.dumps(out), flush=True)
    if pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
