#!/usr/bin/env python3
"""Step pipeline from a rocprofv3 --kernel-trace --memory-copy-trace run (csv, plain or
.gz): per step the ingress H2D, the ingest half (k_stage .. k_decode), the routing /
delivery half (k_marks .. k_post) and the egress D2H, as medians relative to the step's
H2D start, plus how busy each engine was over the traced steps.

usage: pipeline_timeline.py DIR [min_copy_bytes]"""
import csv
import glob
import gzip
import os
import statistics as st
import sys

d = sys.argv[1]
min_bytes = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20


def rows(pattern):
    fs = glob.glob(os.path.join(d, "**", pattern), recursive=True) + \
        glob.glob(os.path.join(d, "**", pattern + ".gz"), recursive=True)
    if not fs:
        return []
    f = fs[0]
    op = gzip.open if f.endswith(".gz") else open
    with op(f, "rt") as fh:
        return list(csv.DictReader(fh))


ING = {"k_stage", "k_frame_scan", "k_scan", "k_decode"}
ks = sorted(rows("*kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
cs = rows("*memory_copy_trace.csv")
h2d, d2h = [], []
for r in cs:
    size = r.get("Bytes") or r.get("Size")
    span_ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    # (no size column in this rocprofv3 version: a payload copy is one longer than 20 us)
    if (int(size) < min_bytes) if size else span_ns < 20000:
        continue
    kind = (r.get("Direction") or r.get("Kind") or "").upper()
    span = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    if "HOST_TO_DEVICE" in kind or "H2D" in kind or "HOSTTODEVICE" in kind:
        h2d.append(span)
    elif "DEVICE_TO_HOST" in kind or "D2H" in kind or "DEVICETOHOST" in kind:
        d2h.append(span)
h2d.sort()
d2h.sort()

steps, cur = [], None
for r in ks:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
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
steps = [x for x in steps if x["rest"]]


def last_before(spans, t):
    best = None
    for a, b in spans:
        if b <= t:
            best = (a, b)
        else:
            break
    return best


def first_after(spans, t):
    for a, b in spans:
        if a >= t:
            return (a, b)
    return None


out = []
for x in steps:
    hh = last_before(h2d, x["ing"][0])
    dd = first_after(d2h, x["rest"][1])
    t0 = hh[0] if hh else x["ing"][0]
    out.append(dict(h2d=(hh[0] - t0, hh[1] - t0) if hh else None, ing=(x["ing"][0] - t0, x["ing"][1] - t0),
                    rest=(x["rest"][0] - t0, x["rest"][1] - t0),
                    d2h=(dd[0] - t0, dd[1] - t0) if dd else None, t0=t0))
out = out[5:-2] if len(out) > 10 else out
if not out:
    print("no steps found")
    sys.exit(0)


def med(key, i):
    v = [o[key][i] / 1e3 for o in out if o[key] is not None]
    return st.median(v) if v else float("nan")


print(f"steps {len(out)}  (us from the step's ingress H2D start; median)")
for k in ("h2d", "ing", "rest", "d2h"):
    print(f"  {k:5s} {med(k, 0):8.1f} .. {med(k, 1):8.1f}")
per = [(b["t0"] - a["t0"]) / 1e3 for a, b in zip(out, out[1:])]
print(f"  step period (H2D start to H2D start): median {st.median(per):.1f} us")
lo, hi = out[0]["t0"], out[-1]["t0"]
for name, spans in (("H2D", h2d), ("D2H", d2h)):
    busy = sum(min(b, hi) - max(a, lo) for a, b in spans if b > lo and a < hi)
    print(f"  {name} engine busy {100.0 * busy / max(1, hi - lo):.0f}% of the traced steps")
kb = sum(min(int(r["End_Timestamp"]), hi) - max(int(r["Start_Timestamp"]), lo) for r in ks
         if int(r["End_Timestamp"]) > lo and int(r["Start_Timestamp"]) < hi)
print(f"  kernels (sum of durations) {100.0 * kb / max(1, hi - lo):.0f}% of the traced steps")
ovl = [max(0, min(a["rest"][1] + a["t0"], b["ing"][1] + b["t0"]) - max(a["rest"][0] + a["t0"], b["ing"][0] + b["t0"])) / 1e3
       for a, b in zip(out, out[1:])]
print(f"  step t+1 ingest overlapping step t routing half: median {st.median(ovl):.1f} us")
