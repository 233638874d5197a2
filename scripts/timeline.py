"""Per-step timeline from a rocprofv3 kernel + memory-copy trace (scripts/prof_timeline.sh)."""
import csv
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_tl"
k = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
k.sort(key=lambda r: int(r["Start_Timestamp"]))
preps = [int(r["Start_Timestamp"]) for r in k if r["Kernel_Name"].startswith("k_prep")]
t0, t1 = preps[-4], preps[-2]
ev = []
for r in k:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if t0 <= s < t1:
        ev.append((s - t0, e - s, "q" + r["Queue_Id"], r["Kernel_Name"][:44]))
mp = os.path.join(d, "run_memory_copy_trace.csv")
if os.path.exists(mp):
    for r in csv.DictReader(open(mp)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 - 600000 <= s < t1 and e - s > 20000:
            ev.append((s - t0, e - s, "copy", r["Direction"]))
busy = sum(x[1] for x in ev if x[2] != "copy" and not x[3].startswith("__amd") and x[0] >= 0)
print(f"2 steps span {(t1 - t0) / 1000:.1f} us; compute kernel busy {busy / 1000:.1f} us")
for s, dur, q, name in sorted(ev):
    print(f"{s / 1000:9.1f} {dur / 1000:8.1f} {q:5s} {name}")
