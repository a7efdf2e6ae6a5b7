#!/usr/bin/env python3
"""Timeline of a rocprofv3 kernel trace: for the last (timed) renderLoop of a
bench run, wall time vs. summed kernel time per kernel, and how much of the
wall time has 0 / 1 / 2+ trace kernels (k_trace_*) running."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "pt::" in r["Kernel_Name"]]
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", ""))
          for r in rows]
    ev.sort()
    # the timed region: after the last k_zero (clearImage) before the final launches
    zs = [i for i, e in enumerate(ev) if "k_zero" in e[2]]
    ev = ev[zs[-1] + 1:] if zs else ev
    t0, t1 = min(e[0] for e in ev), max(e[1] for e in ev)
    wall = t1 - t0
    per = defaultdict(lambda: [0, 0])
    for s, e, n in ev:
        per[n][0] += e - s
        per[n][1] += 1
    print(f"wall {wall / 1e6:.3f} ms, {len(ev)} launches")
    for n, (t, c) in sorted(per.items(), key=lambda x: -x[1][0]):
        print(f"  {n:40s} {c:6d} launches  sum {t / 1e6:9.3f} ms  avg {t / c / 1e3:8.1f} us")
    # concurrency of trace kernels and of all kernels
    for label, pred in (("trace", lambda n: "k_trace_gf" in n or "k_trace_bvh" in n), ("any", lambda n: True)):
        pts = []
        for s, e, n in ev:
            if pred(n):
                pts.append((s, 1)); pts.append((e, -1))
        pts.sort()
        hist = defaultdict(int)
        cur, last = 0, t0
        for t, dlt in pts:
            hist[min(cur, 4)] += t - last
            cur += dlt
            last = t
        hist[0] += t1 - last
        print(f"  {label} kernels running: " + ", ".join(f"{k}{'+' if k == 4 else ''}: {v / wall * 100:.1f}%"
                                                      for k, v in sorted(hist.items())))


if __name__ == "__main__":
    main(sys.argv[1])
