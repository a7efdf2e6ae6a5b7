#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into
profiles/pmc_latest.json (read by bench.py for roofline.traffic).

    python scripts/pmc_summary.py WORKLOAD_KEY FETCH_DIR WRITE_DIR [OUT_JSON]
    python scripts/pmc_summary.py sq WORKLOAD_KEY SQ_DIR [TAG [OUT_JSON]]
    python scripts/pmc_summary.py cycles WORKLOAD_KEY SQ_DIR [TAG [OUT_JSON]]
      (the wave-cycle pass: SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_WAIT_INST_ANY,
      SQ_ACTIVE_INST_ANY, SQ_INSTS_VALU, SQ_THREAD_CYCLES_VALU per trace launch,
      main and tail launches apart; TAG "_cycles_p1" or "_cycles")
      (TAG "_sq": the bench's pipelines, for the whole-job issue rate; "_sq_p1": one
      pipeline, matching bench.py's per-kernel roofline pass)

The iteration count of an SQ pass is the number of first-bounce dispatches it
counted (k_bounce<true, ...>: one per iteration of Renderer.cpp:582-644's loop,
warmup, timed steps and any full-spp render alike), never a number passed in:
round 4 divided a 265-iteration pass by 9 and published an issue fraction of 10.

Per MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KB; on gfx950
FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (the doubling is exact
for the 16-B/lane ray-state streams and an over-estimate for the scattered
scene gathers; raw values are kept alongside).  The two counters come from
separate passes (FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = {
    "k_bounce<false, 2,": "k_bounce<false,grid_fast>",
    "k_bounce<true, 2,": "k_bounce<true,grid_fast>",
    "k_bounce<false, 1,": "k_bounce<false,bvh>",
    "k_bounce<false, 0,": "k_bounce<false,grid>",
    "k_bounce<true, 1,": "k_bounce<true,bvh>",
    "k_bounce<true, 0,": "k_bounce<true,grid>",
    "k_scan": "k_scan",
    "k_trace_bvh<": "k_trace_bvh",
    "k_trace_gf<": "k_trace_gf",
    "k_trace_deferred": "k_trace_deferred",
    "k_bounce<false, 3,": "k_bounce<false,hitbuf>",
    "k_sort_hist": "k_sort_hist",
    "k_sort_prefix": "k_sort_prefix",
    "k_sort_scatter": "k_sort_scatter",
    "k_merge": "k_merge",
    "k_primary": "k_primary",
}


def read_counter(d, counter):
    per = defaultdict(list)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                for k, short in KERNELS.items():
                    if k in name:
                        per[short].append(float(row["Counter_Value"]))
    return per


def counted_iterations(per):
    """Iterations a counter pass ran: its first-bounce (k_bounce<true, ...>)
    dispatches, one per iteration."""
    return max((len(v) for k, v in per.items() if k.startswith("k_bounce<true,")), default=0)


def main_sq(key, sq_dir, tag="_sq", out=None):
    """SQ_INSTS_VALU / SQ_INSTS_SALU pass (wave-level instruction counts, chip
    totals per dispatch): per-kernel counts per launch, and the total of the
    renderer's kernels per iteration, over the iterations the pass counted
    (first-bounce dispatches).  bench.py turns these into an issue roofline."""
    out = out or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_latest.json")
    valu = read_counter(sq_dir, "SQ_INSTS_VALU")
    salu = read_counter(sq_dir, "SQ_INSTS_SALU")
    iterations = max(counted_iterations(valu), counted_iterations(salu))
    if iterations <= 0:
        raise SystemExit(f"pmc_summary: no first-bounce dispatch counted under {sq_dir}")
    per = {}
    tot_v = tot_s = 0.0
    for k in set(valu) | set(salu):
        v, sa = valu.get(k, []), salu.get(k, [])
        per[k] = {"valu_insts_per_launch": sum(v) / max(len(v), 1), "salu_insts_per_launch": sum(sa) / max(len(sa), 1),
                  "launches": max(len(v), len(sa))}
        if k != "k_primary":
            tot_v += sum(v)
            tot_s += sum(sa)
    data = {}
    if os.path.exists(out):
        with open(out) as fh:
            data = json.load(fh)
    data.setdefault(key, {})[tag] = {"iterations": iterations, "valu_insts_per_iteration": tot_v / iterations,
                                       "salu_insts_per_iteration": tot_s / iterations, "kernels": per}
    with open(out, "w") as fh:
        json.dump(data, fh, indent=1, sort_keys=True)
    print(json.dumps(data[key][tag], indent=1))


CYCLE_COUNTERS = ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                  "SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_INSTS_VALU")


def read_trace_launches(d):
    """Per-counter values of the trace kernels, keyed by the launch kind:
    'main' (k_trace_gf/k_trace_bvh<..., false>, the bounce's persistent trace) and
    'tail' (<..., true>: drain continuations and walk hand-ons)."""
    per = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if "k_trace_gf<" not in name and "k_trace_bvh<" not in name:
                    continue
                kind = "tail" if ", true>" in name else "main"
                kern = "k_trace_gf" if "k_trace_gf<" in name else "k_trace_bvh"
                per[f"{kern}.{kind}"][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return per


def main_cycles(key, sq_dir, tag="_cycles_p1", out=None):
    """Wave-cycle split of the trace launches: the share of wave cycles waiting
    on memory (SQ_WAIT_ANY), stalled on issue (SQ_WAIT_INST_ANY) and issuing
    (SQ_ACTIVE_INST_ANY), and the active lanes per VALU instruction
    (SQ_THREAD_CYCLES_VALU / SQ_INSTS_VALU, one wave64 instruction = 64 lane slots)."""
    out = out or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_latest.json")
    per = read_trace_launches(sq_dir)
    res = {}
    for k, cs in per.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items() if v}
        cyc = avg.get("SQ_WAVE_CYCLES", 0.0)
        e = {"launches": max(len(v) for v in cs.values()), **{c.lower() + "_per_launch": avg[c] for c in avg}}
        if cyc > 0:
            for c, name in (("SQ_WAIT_ANY", "wait_share"), ("SQ_WAIT_INST_ANY", "issue_stall_share"),
                            ("SQ_ACTIVE_INST_ANY", "active_share")):
                if c in avg:
                    e[name] = avg[c] / cyc
        if avg.get("SQ_INSTS_VALU", 0) > 0 and "SQ_THREAD_CYCLES_VALU" in avg:
            e["lanes_per_valu"] = avg["SQ_THREAD_CYCLES_VALU"] / avg["SQ_INSTS_VALU"]
        res[k] = e
    if not res:
        raise SystemExit(f"pmc_summary: no trace launch counted under {sq_dir}")
    data = {}
    if os.path.exists(out):
        with open(out) as fh:
            data = json.load(fh)
    data.setdefault(key, {})[tag] = res
    with open(out, "w") as fh:
        json.dump(data, fh, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1))


def main(key, fetch_dir, write_dir, out=None):
    out = out or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_latest.json")
    fetch = read_counter(fetch_dir, "FETCH_SIZE")
    write = read_counter(write_dir, "WRITE_SIZE")
    res = {}
    for k in set(fetch) | set(write):
        f = fetch.get(k, [])
        w = write.get(k, [])
        if not f or not w:
            continue
        fa = sum(f) / len(f)
        wa = sum(w) / len(w)
        res[k] = {"fetch_kb_per_launch": fa, "write_kb_per_launch": wa, "launches": len(f),
                  "hbm_bytes_per_launch": (2.0 * fa + wa) * 1024.0}
    data = {}
    if os.path.exists(out):
        with open(out) as fh:
            data = json.load(fh)
    data.setdefault(key, {}).update(res)
    with open(out, "w") as fh:
        json.dump(data, fh, indent=1, sort_keys=True)
    print(json.dumps({key: res}, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "sq":
        main_sq(*sys.argv[2:])
    elif sys.argv[1] == "cycles":
        main_cycles(*sys.argv[2:])
    else:
        main(*sys.argv[1:])
