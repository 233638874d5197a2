#!/usr/bin/env python3
"""Per-kernel duration and launch gap of the data-plane step from a rocprofv3 kernel
trace (csv): steps are split at k_stage; for every position in the step, the median
duration, the median gap since the previous kernel of the step ended, and the median
step span (k_stage start -> last kernel end).  usage: step_gaps.py DIR [skip_steps]"""
import csv
import glob
import os
import statistics as st
import sys


def main(d, skip=5):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], None
    for r in rows:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if not n.startswith("k_") and "k_scan" not in n and "k_rs_" not in n:
            continue
        if n.startswith("k_stage"):
            cur = []
            steps.append(cur)
        if cur is not None:
            cur.append((n, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    steps = steps[skip:-1] if len(steps) > skip + 1 else steps
    if not steps:
        print("no steps")
        return
    L = st.median([len(s) for s in steps])
    steps = [s for s in steps if len(s) == L]
    print(f"{len(steps)} steps of {L} kernels")
    tot_d = tot_g = 0.0
    print("pos,kernel,dur_us,gap_us")
    for i in range(int(L)):
        durs = [(s[i][2] - s[i][1]) / 1e3 for s in steps]
        gaps = [((s[i][1] - s[i - 1][2]) / 1e3) if i else 0.0 for s in steps]
        md, mg = st.median(durs), st.median(gaps)
        tot_d += md
        tot_g += mg
        print(f"{i},{steps[0][i][0]},{md:.2f},{mg:.2f}")
    span = st.median([(s[-1][2] - s[0][1]) / 1e3 for s in steps])
    print(f"sum_dur_us,{tot_d:.1f}\nsum_gap_us,{tot_g:.1f}\nspan_us,{span:.1f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5)
