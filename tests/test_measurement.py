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
    the once-per-renderer k_primary."""
    m = _pmc_summary()
    gf = "void pt::k_trace_gf<64, 9, false>(pt::KParams, int, int)"
    rows = [
        {"Kernel_Name": gf, "Counter_Name": "SQ_INSTS_VALU", "Counter_Value": 100.0},
        {"Kernel_Name": gf, "Counter_Name": "SQ_INSTS_VALU", "Counter_Value": 300.0},
        {"Kernel_Name": gf, "Counter_Name": "SQ_INSTS_SALU", "Counter_Value": 50.0},
        {"Kernel_Name": gf, "Counter_Name": "SQ_INSTS_SALU", "Counter_Value": 70.0},
        {"Kernel_Name": "void pt::k_primary<2>(pt::KParams)", "Counter_Name": "SQ_INSTS_VALU", "Counter_Value": 1e6},
        {"Kernel_Name": "void pt::k_primary<2>(pt::KParams)", "Counter_Name": "SQ_INSTS_SALU", "Counter_Value": 1e6},
        {"Kernel_Name": "pt::k_scan(pt::KParams, int)", "Counter_Name": "SQ_INSTS_VALU", "Counter_Value": 20.0},
        {"Kernel_Name": "pt::k_scan(pt::KParams, int)", "Counter_Name": "SQ_INSTS_SALU", "Counter_Value": 10.0},
    ]
    _write_counters(str(tmp_path / "sq"), rows)
    out = str(tmp_path / "pmc.json")
    with open(out, "w") as f:      # an existing FETCH/WRITE entry for the key survives
        json.dump({"w": {"k_trace_gf": {"hbm_bytes_per_launch": 5.0}}}, f)
    m.main_sq("w", str(tmp_path / "sq"), 2, "_sq", out)
    d = json.load(open(out))["w"]
    assert d["k_trace_gf"]["hbm_bytes_per_launch"] == 5.0
    sq = d["_sq"]
    assert sq["kernels"]["k_trace_gf"]["valu_insts_per_launch"] == 200.0
    assert sq["kernels"]["k_trace_gf"]["launches"] == 2
    assert sq["valu_insts_per_iteration"] == (400.0 + 20.0) / 2
    assert sq["salu_insts_per_iteration"] == (120.0 + 10.0) / 2


def test_committed_pmc_summary_has_bench_keys():
    """bench.py's roofline.traffic and issue_roofline read these entries for the
    default workload (both accelerations)."""
    d = json.load(open(os.path.join(ROOT, "profiles", "pmc_latest.json")))
    for accel, kern in (("grid_fast", "k_trace_gf"), ("bvh", "k_trace_bvh")):
        e = d[f"{accel}_100000_1280x1024_b8"]
        assert e[kern]["hbm_bytes_per_launch"] > 0
        assert e["_sq"]["valu_insts_per_iteration"] > 0
        assert e["_sq_p1"]["kernels"][kern]["valu_insts_per_launch"] > 0


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
    """--gpus 2 without a launcher starts two ranks itself; here (no GPU) both
    fail, and the parent reports the failure with a non-zero exit instead of
    hanging or printing a result line."""
    p = _run_bench(["--gpus", "2", "--dist-backend", "gloo", "--steps", "1", "--warmup", "0", "--targets=",
                    "--alt-accel=", "--no-cpu-baseline", "--no-full-runs", "--no-profile"], {})
    assert p.returncode != 0
    assert "exited with" in p.stderr
    assert '"metric"' not in p.stdout
