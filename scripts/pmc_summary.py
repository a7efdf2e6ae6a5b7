#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into
profiles/pmc_latest.json (read by bench.py for roofline.traffic).

    python scripts/pmc_summary.py WORKLOAD_KEY FETCH_DIR WRITE_DIR [OUT_JSON]

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
    data[key] = res
    with open(out, "w") as fh:
        json.dump(data, fh, indent=1, sort_keys=True)
    print(json.dumps({key: res}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
