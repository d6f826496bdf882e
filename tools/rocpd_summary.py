#!/usr/bin/env python3
"""Kernel-duration summary of a rocprofv3 rocpd database (ROCm 7 writes
<name>_results.db by default): per (kernel, grid size) the dispatch count and
average / min / max / total duration in microseconds — what
`rocprofv3 --kernel-trace --stats` reports, split by launch shape so that
one tool's size sweep separates into its sizes.

With --segments, consecutive dispatches of one (kernel, grid) in time order
form one row each — a sweep tool's phases, in the order it ran them.

usage: rocpd_summary.py RESULTS_DB [OUT_CSV] [--by-name | --segments]"""
import csv
import os
import sqlite3
import sys


def short(name):
    name = name.replace("gloo_amd::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    return name.split("(", 1)[0].split("<", 1)[0].replace("void ", "")


def main():
    if len(sys.argv) < 2 or sys.argv[1].startswith("-") or not os.path.isfile(sys.argv[1]):
        sys.exit(__doc__)  # never let sqlite3.connect create a file named after a flag
    db = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else None
    by_name = "--by-name" in sys.argv
    con = sqlite3.connect(db)
    if "--segments" in sys.argv:
        rows = con.execute("select name, grid_x, workgroup_x, start, end from kernels order by start").fetchall()
        segs = []
        for name, g, wg, b, e in rows:
            if segs and segs[-1][0] == (name, g, wg):
                segs[-1][1].append(e - b)
            else:
                segs.append([(name, g, wg), [e - b]])
        w = csv.writer(open(out, "w", newline="") if out else sys.stdout)
        w.writerow(["segment", "kernel", "grid_threads", "workgroup", "calls", "avg_us", "median_us", "min_us", "max_us"])
        for i, ((name, g, wg), d) in enumerate(segs):
            d = sorted(d)
            w.writerow([i, short(name), g, wg, len(d), round(sum(d) / len(d) / 1e3, 3), round(d[len(d) // 2] / 1e3, 3),
                        round(d[0] / 1e3, 3), round(d[-1] / 1e3, 3)])
        return
    key = "name" if by_name else "name, grid_x, workgroup_x"
    rows = con.execute(f"select {key}, count(*), avg(end - start), min(end - start), max(end - start), "
                       f"sum(end - start) from kernels group by {key} order by sum(end - start) desc").fetchall()
    hdr = ["kernel"] + ([] if by_name else ["grid_threads", "workgroup"]) + \
          ["calls", "avg_us", "min_us", "max_us", "total_us"]
    table = []
    for r in rows:
        k = [short(r[0])] + list(r[1:-5])
        table.append(k + [r[-5]] + [round(v / 1e3, 3) for v in r[-4:]])
    w = csv.writer(open(out, "w", newline="") if out else sys.stdout)
    w.writerow(hdr)
    w.writerows(table)


if __name__ == "__main__":
    main()
