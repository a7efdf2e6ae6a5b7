"""Measurement plumbing on CPU: the PMC summariser (scripts/pmc_summary.py)
and the committed counter summary that bench.py's roofline objects read."""
import csv
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _pmc_summary():
    spec = importlib.util.spec_from_file_location("pmc_summary", os.path.join(ROOT, "scripts", "pmc_summary.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _write_counters(d, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def test_sq_summary_per_iteration(tmp_path):
    """VALU/SALU counts per launch per kernel; the per-iteration total leaves out
    the once-per-renderer k_primary and divides by the iterations the pass
    counted (its first-bounce dispatches)."""
    m = _pmc_summary()
    gf = "void pt::k_trace_gf<64, 9, false>(pt::KParams, int, int)"
    first = "void pt::k_bounce<true, 2, 64>(pt::KParams, int, int)"
    rows = [
        {"Kernel_Name": gf, "Counter_Name": "SQ_INSTS_VALU", "Counter_Value": 100.0},
        {"Kernel_Name": gf, "Counter_Name": "SQ_INSTS_VALU", "Counter_Value": 300.0},
        {"Kernel_Name": gf, "Counter_Name": "SQ_INSTS_SALU", "Counter_Value": 50.0},
        {"Kernel_Name": gf, "Counter_Name": "SQ_INSTS_SALU", "Counter_Value": 70.0},
        {"Kernel_Name": "void pt::k_primary<2>(pt::KParams)", "Counter_Name": "SQ_INSTS_VALU", "Counter_Value": 1e6},
        {"Kernel_Name": "void pt::k_primary<2>(pt::KParams)", "Counter_Name": "SQ_INSTS_SALU", "Counter_Value": 1e6},
        {"Kernel_Name": "pt::k_scan(pt::KParams, int)", "Counter_Name": "SQ_INSTS_VALU", "Counter_Value": 20.0},
        {"Kernel_Name": "pt::k_scan(pt::KParams, int)", "Counter_Name": "SQ_INSTS_SALU", "Counter_Value": 10.0},
    ] + [{"Kernel_Name": first, "Counter_Name": c, "Counter_Value": 0.0}
         for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU") for _ in range(2)]
    _write_counters(str(tmp_path / "sq"), rows)
    out = str(tmp_path / "pmc.json")
    with open(out, "w") as f:      # an existing FETCH/WRITE entry for the key survives
        json.dump({"w": {"k_trace_gf": {"hbm_bytes_per_launch": 5.0}}}, f)
    m.main_sq("w", str(tmp_path / "sq"), "_sq", out)
    d = json.load(open(out))["w"]
    assert d["k_trace_gf"]["hbm_bytes_per_launch"] == 5.0
    sq = d["_sq"]
    assert sq["iterations"] == 2
    assert sq["kernels"]["k_trace_gf"]["valu_insts_per_launch"] == 200.0
    assert sq["kernels"]["k_trace_gf"]["launches"] == 2
    assert sq["valu_insts_per_iteration"] == (400.0 + 20.0) / 2
    assert sq["salu_insts_per_iteration"] == (120.0 + 10.0) / 2


def test_sq_summary_counts_every_iteration_the_pass_ran(tmp_path):
    """Round 4's pass ran 1 warmup + 8 steps + a 256-spp full render = 265
    iterations and was divided by a hard-coded 9.  The summary now takes the
    iteration count from the 265 first-bounce dispatches themselves."""
    m = _pmc_summary()
    first = "void pt::k_bounce<true, 2, 64>(pt::KParams, int, int)"
    gf = "void pt::k_trace_gf<64, 25, false>(pt::KParams, int, int)"
    iters, bounces, v_launch = 265, 7, 146.0e6
    rows = [{"Kernel_Name": first, "Counter_Name": "SQ_INSTS_VALU", "Counter_Value": 8.7e6} for _ in range(iters)]
    rows += [{"Kernel_Name": gf, "Counter_Name": "SQ_INSTS_VALU", "Counter_Value": v_launch}
             for _ in range(iters * bounces)]
    rows += [{"Kernel_Name": first, "Counter_Name": "SQ_INSTS_SALU", "Counter_Value": 1.0} for _ in range(iters)]
    _write_counters(str(tmp_path / "sq"), rows)
    out = str(tmp_path / "pmc.json")
    m.main_sq("k", str(tmp_path / "sq"), "_sq", out)
    sq = json.load(open(out))["k"]["_sq"]
    assert sq["iterations"] == iters
    assert abs(sq["valu_insts_per_iteration"] - (8.7e6 + bounces * v_launch)) < 1.0
    # and an issue fraction from it stays below 1 at the round-4 step time
    b = _bench()
    assert sq["valu_insts_per_iteration"] / 1.896e-3 / 1e9 / b.VALU_PEAK_G < 1.0


def test_sq_summary_refuses_a_pass_without_iterations(tmp_path):
    import pytest
    m = _pmc_summary()
    _write_counters(str(tmp_path / "sq"), [{"Kernel_Name": "pt::k_scan(pt::KParams, int)",
                                            "Counter_Name": "SQ_INSTS_VALU", "Counter_Value": 1.0}])
    with pytest.raises(SystemExit):
        m.main_sq("k", str(tmp_path / "sq"), "_sq", str(tmp_path / "o.json"))


def test_cycles_summary_splits_main_and_tail(tmp_path):
    m = _pmc_summary()
    main = "void pt::k_trace_gf<64, 9, false>(pt::KParams, int, int)"
    tail = "void pt::k_trace_gf<64, 9, true>(pt::KParams, int, int)"
    rows = []
    for name, wait, lanes in ((main, 50.0, 24.0), (tail, 80.0, 8.0)):
        rows += [{"Kernel_Name": name, "Counter_Name": "SQ_WAVE_CYCLES", "Counter_Value": 100.0},
                 {"Kernel_Name": name, "Counter_Name": "SQ_WAIT_ANY", "Counter_Value": wait},
                 {"Kernel_Name": name, "Counter_Name": "SQ_INSTS_VALU", "Counter_Value": 10.0},
                 {"Kernel_Name": name, "Counter_Name": "SQ_THREAD_CYCLES_VALU", "Counter_Value": 10.0 * lanes}]
    _write_counters(str(tmp_path / "c"), rows)
    out = str(tmp_path / "pmc.json")
    m.main_cycles("k", str(tmp_path / "c"), "_cycles", out)
    d = json.load(open(out))["k"]["_cycles"]
    assert d["k_trace_gf.main"]["wait_share"] == 0.5 and d["k_trace_gf.main"]["lanes_per_valu"] == 24.0
    assert d["k_trace_gf.tail"]["wait_share"] == 0.8 and d["k_trace_gf.tail"]["lanes_per_valu"] == 8.0


def test_bench_never_publishes_a_fraction_above_one():
    b = _bench()
    line = {"roofline": {"frac": 0.0087, "issue": {"frac": 0.22}},
            "issue_roofline": {"job": {"frac": 10.45}},
            "targets": {"configs4": {"roofline": {"frac": float("nan")}}}}
    bad = b.bound_fracs(line)
    assert sorted(bad) == ["line.issue_roofline.job", "line.targets.configs4.roofline"]
    assert line["issue_roofline"]["job"]["frac"] is None and "error" in line["issue_roofline"]["job"]
    assert line["targets"]["configs4"]["roofline"]["frac"] is None
    assert line["roofline"]["frac"] == 0.0087 and line["roofline"]["issue"]["frac"] == 0.22


def test_committed_pmc_summary_has_bench_keys():
    """bench.py's roofline.traffic and issue_roofline read these entries for the
    default workload (both accelerations); every SQ entry divides by the
    iterations its pass counted, and the fractions it implies stay below 1."""
    d = json.load(open(os.path.join(ROOT, "profiles", "pmc_latest.json")))
    for accel, kern in (("grid_fast", "k_trace_gf"), ("bvh", "k_trace_bvh")):
        e = d[f"{accel}_100000_1280x1024_b8"]
        assert e[kern]["hbm_bytes_per_launch"] > 0
        assert e["_sq"]["valu_insts_per_iteration"] > 0
        assert e["_sq_p1"]["kernels"][kern]["valu_insts_per_launch"] > 0
        for tag in ("_sq", "_sq_p1"):
            per_it = e[tag]["valu_insts_per_iteration"]
            launches = e[tag]["kernels"][kern]["launches"]
            assert launches % e[tag]["iterations"] == 0          # whole bounces per iteration
            # at most a few G wave-instructions per 1280x1024 sample: a mis-divided pass is 30x that
            assert per_it < 2.0e9
    cyc = d["grid_fast_100000_1280x1024_b8"]["_cycles_p1"]["k_trace_gf.main"]
    assert 0 < cyc["wait_share"] < 1 and 0 < cyc["lanes_per_valu"] <= 64


def _bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_bench_rates_and_roofline_bytes():
    """bench.py's arithmetic: segment rate with and without the cached primary
    bounce, samples/s over all ranks, and the trace's algorithmic bytes per step
    (52 B per segment entering bounce >= 1)."""
    b = _bench()
    res = {"elapsed": 2.0, "seg": 8.0e9, "seg_primary": 2.0e9}
    r = b.rates(res, K=100, npix=1000, world=2)
    assert r["value"] == 4000.0 and r["traced_mrays_per_sec"] == 3000.0
    assert r["ms_per_step"] == 20.0 and r["samples_per_sec"] == 2 * 100 * 1000 / 2.0
    assert b.trace_bytes_per_step([10, 6, 4, 0], K=2) == 52.0 * 10 / 2
    assert b.VALU_PEAK_G == 256 * 4 * 2.4 / 2


def test_bench_workload_labels():
    b = _bench()
    import argparse
    a = argparse.Namespace(scene="", ntri=100_000, width=1280, height=1024, bounces=8, metallic=False)
    assert b.workload_name(a).startswith("configs[1]")
    a.ntri = 1_000_000
    assert b.workload_name(a).startswith("north_star target")
    a.ntri, a.bounces = 10_000_000, 16
    assert b.workload_name(a).startswith("configs[4]")


def test_bench_full_rates():
    """The full-spp render: spp iterations over all ranks in `seconds`."""
    b = _bench()
    res = {"full": {"spp": 256, "elapsed": 0.5, "seg": 1.0e9, "seg_primary": 2.5e8, "img_ok": True}}
    f = b.full_rates(res, npix=1000)
    assert f["spp"] == 256 and f["value"] == 2000.0 and f["traced_mrays_per_sec"] == 1500.0
    assert f["samples_per_sec"] == 256 * 1000 / 0.5
    assert b.full_rates({}, 1000) is None
    assert b.SPP == {"configs1": 256, "target_1m": 1024, "configs2": 1024, "configs4": 4096}


def test_bench_cpu_share_honours_the_pool_share(monkeypatch):
    b = _bench()
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    n, why = b.host_cpu_share()
    assert n == min(3, len(os.sched_getaffinity(0))) and "OMP_NUM_THREADS 3" in why
    monkeypatch.delenv("OMP_NUM_THREADS")
    n, why = b.host_cpu_share()
    assert n == len(os.sched_getaffinity(0)) or "cgroup" in why


def _run_bench(args, env_extra, timeout=180):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_rejects_world_size_mismatch():
    """Under a launcher the world size must equal --gpus (checked before any GPU call)."""
    p = _run_bench(["--gpus", "3"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "--gpus 3 but the launcher started 2" in p.stderr


def test_bench_spawned_ranks_fail_together():
    """--gpus 2 without a launcher starts two ranks itself; a rank that fails
    (here: a scene file that does not exist, on any host) makes the parent
    report the failure with a non-zero exit instead of hanging or printing a
    result line."""
    p = _run_bench(["--gpus", "2", "--dist-backend", "gloo", "--steps", "1", "--warmup", "0", "--targets=",
                    "--alt-accel=", "--no-cpu-baseline", "--no-full-runs", "--no-profile",
                    "--scene", "/nonexistent/scene.txt"], {})
    assert p.returncode != 0
    assert "exited with" in p.stderr
    assert '"metric"' not in p.stdout


def test_bench_nccl_needs_a_gpu_per_rank():
    """RCCL with more ranks than visible GPUs is refused before init_process_group
    (it would map two ranks onto one device and fail or hang in the rendezvous)."""
    b = _bench()
    assert b.check_backend("nccl", 8, 8) is None and b.check_backend("gloo", 2, 1) is None
    assert "one GPU per rank" in b.check_backend("nccl", 2, 1)
    import torch
    n = torch.cuda.device_count()
    p = _run_bench(["--gpus", str(n + 1), "--dist-backend", "nccl"],
                   {"WORLD_SIZE": str(n + 1), "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": "1"}, timeout=120)
    assert p.returncode != 0 and "one GPU per rank" in p.stderr
