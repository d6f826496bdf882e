#!/usr/bin/env python3
"""Per-launch HBM traffic of the reduce kernel from rocprofv3 --pmc passes.

Collected as MI355X_MICROARCH.md's HBM section prescribes: FETCH_SIZE and
WRITE_SIZE in SEPARATE passes (TCC slots: 3 + 2 > 4), both in KiB; on gfx950
FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane) coalesced
streaming read, so it is doubled; WRITE_SIZE is exact for 16-B streaming stores.

usage: pmc_traffic.py FETCH_CSV WRITE_CSV ELEMENTS OUT_JSON [KERNEL_SUBSTR]
"""
import csv
import json
import statistics
import sys


def per_launch(path, counter, substr):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if substr in r["Kernel_Name"] and r["Counter_Name"] == counter]
    if not vals:
        raise SystemExit(f"no {counter} rows for {substr} in {path}")
    return statistics.median(vals), len(vals)


def main():
    fetch_csv, write_csv, elements, out = sys.argv[1:5]
    substr = sys.argv[5] if len(sys.argv) > 5 else "reduce_vec_kernel"
    elements = int(elements)
    f_kib, nf = per_launch(fetch_csv, "FETCH_SIZE", substr)
    w_kib, nw = per_launch(write_csv, "WRITE_SIZE", substr)
    read_b = 2 * f_kib * 1024          # gfx950 correction: FETCH_SIZE is half
    write_b = w_kib * 1024
    alg = 3 * elements * 4
    res = {"elements": elements, "kernel": substr,
           "fetch_size_kib_raw": f_kib, "write_size_kib": w_kib,
           "hbm_read_bytes_per_launch": int(read_b), "hbm_write_bytes_per_launch": int(write_b),
           "hbm_bytes_per_launch": int(read_b + write_b), "algorithmic_bytes_per_launch": alg,
           "traffic_over_algorithmic": round((read_b + write_b) / alg, 5),
           "dispatches": {"fetch": nf, "write": nw},
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate passes; "
                     "FETCH_SIZE x2 (gfx950 wide-read correction), KiB x1024; median over dispatches"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
