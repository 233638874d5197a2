#!/usr/bin/env python3
"""Mean kernel time of consecutive same-name launch groups of a rocprofv3 kernel trace
(rocpd db): usage parse_trace.py DB [group_size]"""
import glob
import sqlite3
import sys


def main(db, group=50):
    cur = sqlite3.connect(db).cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = [(n.split("(")[0].replace("void ", ""), (e - s) / 1e3)
            for n, s, e in cur.execute(f"select {name}, start, end from kernels order by start")]
    # split each name's launches into runs of `group` in order of appearance
    seen = {}
    for n, t in rows:
        seen.setdefault(n, []).append(t)
    for n, ts in seen.items():
        parts = [ts[i:i + group] for i in range(0, len(ts), group)]
        print(n, " | ".join(f"{sorted(p)[len(p) // 2]:.2f}" for p in parts), "(median us per group of", group, ")")


if __name__ == "__main__":
    db = sys.argv[1]
    if not db.endswith(".db"):
        db = glob.glob(db + "/**/*.db", recursive=True)[0]
    main(db, int(sys.argv[2]) if len(sys.argv) > 2 else 50)
