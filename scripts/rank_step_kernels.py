#!/usr/bin/env python3
"""Kernel time per rank-step from a rocprofv3 rocpd db of bench/world_rehearsal.py (or
bench.py with --world 1): data-plane kernels only (k_*), runtime copies/fills excluded.
Second table: the launch sequence of each graph (split at k_stage = phase A / whole step,
k_import = phase B), mean time per position, so repeated kernels (k_route in phase A and
in phase B) are told apart.
usage: rank_step_kernels.py DB RANK_STEPS [out.csv]"""
import sqlite3
import sys
from collections import defaultdict


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
    # per graph position
    seqs, cur_seq = [], None
    for n, s, e in cur.execute(f"select {name}, start, end from kernels order by start"):
        n = n.split("(")[0].replace("void ", "")
        if "k_" not in n:
            continue
        if n in ("k_stage", "k_import", "k_import_route"):
            cur_seq = []
            seqs.append(cur_seq)
        if cur_seq is not None:
            cur_seq.append((n, (e - s) / 1e3))
    groups = defaultdict(list)
    for sq in seqs:
        groups[tuple(n for n, _ in sq)].append([t for _, t in sq])
    for sig, runs in sorted(groups.items(), key=lambda kv: -len(kv[1])):
        if len(runs) < 2:
            continue
        lines.append("")
        lines.append(f"graph starting {sig[0]} ({len(runs)} runs): position,kernel,mean_us")
        tot = 0.0
        for i, n in enumerate(sig):
            m = sum(r[i] for r in runs) / len(runs)
            tot += m
            lines.append(f"{i},{n},{m:.2f}")
        lines.append(f"TOTAL,{len(sig)},{tot:.2f}")
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]), sys.argv[3] if len(sys.argv) > 3 else None)
