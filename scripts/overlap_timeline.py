#!/usr/bin/env python3
"""Overlap of consecutive steps in a rocprofv3 kernel trace (csv): per step, the ingest
half (k_stage .. k_decode) and the routing/delivery half (k_marks .. k_post); reports how
much of step t+1's ingest ran while step t's second half was still running.
usage: overlap_timeline.py DIR"""
import csv
import glob
import os
import statistics as st
import sys

d = sys.argv[1]
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
ING = {"k_stage", "k_frame_scan", "k_scan", "k_decode"}
steps, cur, half = [], None, None
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
    s, e, q = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "")
    if n == "k_stage":
        cur = {"ing": [s, e], "rest": None}
        steps.append(cur)
    elif cur is None:
        continue
    elif n in ING and cur["rest"] is None:
        cur["ing"][1] = max(cur["ing"][1], e)
    else:
        if cur["rest"] is None:
            cur["rest"] = [s, e]
        cur["rest"][1] = max(cur["rest"][1], e)
steps = [x for x in steps if x["rest"]][5:-1]
ov = []
for a, b in zip(steps, steps[1:]):
    # step b's ingest overlapping step a's second half
    ov.append(max(0, min(a["rest"][1], b["ing"][1]) - max(a["rest"][0], b["ing"][0])) / 1e3)
ing = [(x["ing"][1] - x["ing"][0]) / 1e3 for x in steps]
rest = [(x["rest"][1] - x["rest"][0]) / 1e3 for x in steps]
per = [(b["rest"][1] - a["rest"][1]) / 1e3 for a, b in zip(steps, steps[1:])]
print(f"steps {len(steps)}: ingest half median {st.median(ing):.1f} us, second half {st.median(rest):.1f} us")
print(f"step t+1 ingest overlapping step t second half: median {st.median(ov):.1f} us")
print(f"completion period (second half end to end): median {st.median(per):.1f} us")
