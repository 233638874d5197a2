#!/usr/bin/env python3
"""Kernel time per rank-step from a rocprofv3 rocpd db of bench/world_rehearsal.py (or
bench.py with --world 1): data-plane kernels only (k_*), runtime copies/fills excluded.
usage: rank_step_kernels.py DB RANK_STEPS [out.csv]"""
import sqlite3
import sys


def main(db, rank_steps, out=None):
    cur = sqlite3.connect(db).cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else cols[0])
    rows = cur.execute(f"select {name}, count(*), sum(end-start) from kernels group by {name}").fetchall()
    lines = ["kernel,launches_per_rank_step,us_per_rank_step"]
    tot_us = tot_l = 0.0
    for n, c, s in sorted(rows, key=lambda r: -r[2]):
        n = n.split("(")[0]
        if "k_" not in n:
            continue
        l, us = c / rank_steps, s / 1e3 / rank_steps
        tot_us += us
        tot_l += l
        lines.append(f"{n},{l:.2f},{us:.2f}")
    lines.append(f"TOTAL,{tot_l:.2f},{tot_us:.2f}")
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]), sys.argv[3] if len(sys.argv) > 3 else None)
