#!/usr/bin/env python3
"""Kernel timeline of the last calls in a rocprofv3 --kernel-trace CSV
(tools/latency_trace.sh): the kernels of rank 0's last N calls, each with its
start relative to the call's first kernel, its duration and the gap before it.
A call starts where the gap to the previous kernel exceeds --split µs (the
host synchronises between calls).

usage: trace_timeline.py KERNEL_TRACE_CSV [N=3] [--split 8]"""
import csv
import sys


def short(name):
    name = name.replace("gloo_amd::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    return name.split("(", 1)[0].split("<", 1)[0].replace("void ", "").strip()


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else 3
    split = float(sys.argv[sys.argv.index("--split") + 1]) if "--split" in sys.argv else 8.0
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r.get("Grid_Size", ""))
                   for r in csv.DictReader(open(path))), key=lambda x: x[0])
    rows = [r for r in rows if r[2] != "nop_kernel"]
    calls, cur, prev_end = [], [], None
    for b, e, name, grid in rows:
        if prev_end is not None and (b - prev_end) / 1e3 > split and cur:
            calls.append(cur)
            cur = []
        cur.append((b, e, name, grid))
        prev_end = e if prev_end is None else max(prev_end, e)
    if cur:
        calls.append(cur)
    for call in calls[-n:]:
        t0, last = call[0][0], call[0][0]
        print(f"--- call: {len(call)} kernels, {(max(e for _, e, _, _ in call) - t0) / 1e3:.2f} us first start to last end")
        for b, e, name, grid in call:
            print(f"{name:28s} grid={grid:>8} start={(b - t0) / 1e3:8.2f} dur={(e - b) / 1e3:7.2f} gap={(b - last) / 1e3:6.2f}")
            last = max(last, e)


if __name__ == "__main__":
    main()
