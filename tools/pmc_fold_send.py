#!/usr/bin/env python3
"""Summarise tools/pmc_fold_send.sh: per variant, the median per dispatch of
every counter for the fold kernels (fold_send_kernel when fused, the fold
kernel otherwise) and the copy kernel, beside the algorithmic bytes.

usage: pmc_fold_send.py OUT_DIR COUNT"""
import csv
import glob
import json
import os
import statistics
import sys


def rows(d):
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        yield from csv.DictReader(open(path))


def main():
    out, count = sys.argv[1], int(sys.argv[2])
    half = count // 2 * 4  # bytes of each rank's half
    res = {"count": count, "bytes_per_rank": count * 4,
           "fold_alg_read_bytes": 2 * half, "fold_alg_write_bytes": half,
           "forward_alg_write_bytes": half, "variants": {}}
    for variant in ("fused", "unfused", "coarse"):
        v = {}
        for d in glob.glob(os.path.join(out, f"pmcfs_{variant}_*")):
            per = {}
            for r in rows(d):
                name = r["Kernel_Name"]
                key = ("fold_send" if "fold_send" in name else "fold" if "fold" in name or "multi" in name
                       else "copy" if "copy" in name else None)
                if key is None:
                    continue
                per.setdefault((key, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
            for (key, cn), vals in per.items():
                v.setdefault(key, {})[cn] = {"median": statistics.median(vals), "dispatches": len(vals)}
        for key, c in v.items():
            if "FETCH_SIZE" in c:
                c["read_bytes_fetch_x2"] = int(2 * 1024 * c["FETCH_SIZE"]["median"])
            if "WRITE_SIZE" in c:
                c["write_bytes"] = int(1024 * c["WRITE_SIZE"]["median"])
        res["variants"][variant] = v
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
