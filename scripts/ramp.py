#!/usr/bin/env python3
"""Ramp profile of the timed renderLoop in a rocprofv3 kernel trace: the region
(after the last k_zero) cut into NBINS slices of wall time, and per slice the
average number of running trace kernels (main + tail launches) and of any
kernels, plus the iterations starting (k_bounce<true>) and ending (k_merge) in
it.  Shows how much of a short timed region runs with few iterations in flight.

    python scripts/ramp.py gpurun_out/s1_ktrace [NBINS]
"""
import csv
import glob
import os
import sys


def main(d, nbins=20):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "pt::" in r["Kernel_Name"]]
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r["Kernel_Name"].split("(")[0].replace("void ", "")) for r in rows)
    zs = [i for i, e in enumerate(ev) if "k_zero" in e[2]]
    ev = ev[zs[-1] + 1:] if zs else ev
    t0, t1 = min(e[0] for e in ev), max(e[1] for e in ev)
    w = (t1 - t0) / nbins
    print(f"timed region {(t1 - t0) / 1e6:.3f} ms in {nbins} slices of {w / 1e3:.1f} us")
    print(" slice   trace_kernels  any_kernels  iters_started  iters_merged")
    for b in range(nbins):
        lo, hi = t0 + b * w, t0 + (b + 1) * w
        tr = an = 0.0
        st = mg = 0
        for s, e, n in ev:
            ov = max(0.0, min(e, hi) - max(s, lo))
            an += ov
            if "k_trace_gf" in n or "k_trace_bvh" in n:
                tr += ov
            if lo <= s < hi and "k_bounce<true" in n:
                st += 1
            if lo <= e < hi and "k_merge" in n:
                mg += 1
        print(f" {b:5d}   {tr / w:13.2f}  {an / w:11.2f}  {st:13d}  {mg:12d}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
