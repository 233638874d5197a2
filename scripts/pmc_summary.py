#!/usr/bin/env python3
"""Mean counter value per dispatch, per kernel, from a rocprofv3 --pmc csv output dir
(…counter_collection.csv).  usage: pmc_summary.py DIR"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(lambda: [0.0, 0])
    disp = defaultdict(set)
    ctrs = []
    for f in files:
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "").split("(")[0].replace("void ", "")
            if "k_" not in k:
                continue
            c = row["Counter_Name"]
            if c not in ctrs:
                ctrs.append(c)
            a = acc[(k, c)]
            a[0] += float(row["Counter_Value"])
            a[1] += 1
            disp[k].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
    kernels = sorted(disp, key=lambda k: -acc[(k, ctrs[0])][0] / max(1, acc[(k, ctrs[0])][1]) if ctrs else 0)
    print("kernel,dispatches," + ",".join(ctrs))
    for k in kernels:
        vals = []
        for c in ctrs:
            s, n = acc[(k, c)]
            vals.append(f"{s / len(disp[k]):.0f}" if disp[k] else "")
        print(f"{k},{len(disp[k])}," + ",".join(vals))


if __name__ == "__main__":
    main(sys.argv[1])
