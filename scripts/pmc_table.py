#!/usr/bin/env python3
"""Average per-dispatch PMC values per kernel from rocprofv3 counter CSVs."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(*dirs):
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                name = row["Kernel_Name"]
                if "pt::" not in name:
                    continue
                short = name.split("(")[0].replace("void ", "")
                acc[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} avg {sum(v) / len(v):16.1f}  n={len(v)}")


if __name__ == "__main__":
    main(*sys.argv[1:])
