#!/usr/bin/env python3
"""Per-kernel stats (calls, total/avg/max us, % of total) from a rocprofv3 rocpd SQLite db."""
import sqlite3
import sys


def main(db, out=None):
    cur = sqlite3.connect(db).cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else cols[0])
    rows = cur.execute(f"select {name}, count(*), sum(end-start), avg(end-start), max(end-start) from kernels "
                       f"group by {name} order by sum(end-start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    lines = ["kernel,calls,total_us,avg_us,max_us,pct"]
    for n, c, s, a, m in rows:
        lines.append(f"{n.split('(')[0]},{c},{s / 1e3:.1f},{a / 1e3:.2f},{m / 1e3:.2f},{100.0 * s / tot:.1f}")
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main(*sys.argv[1:])
