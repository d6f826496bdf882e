"""Runs oracle/_ref/newstyle_test on golden cases and prints the verdicts
(the body of tests/test_gloo_collectives.py, for quick diagnosis).

  python tools/newstyle_case.py MODE [KEY_SUBSTRING ...]
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gloo_collectives as t  # noqa: E402


def run(src, case, mode, timeout=110):
    z = np.load(t.SCHED if src == "sched" else t.NEWSTYLE)
    parts = case.split("/")
    kind = {"allreduce_new": "ring", "bcube": "bcube", "reduce": "reduce"}[parts[0]]
    op, dtype, P = parts[1], parts[2], int(parts[3][1:])
    init, want = z[case + "/init"], z[case + "/out"]
    if kind == "reduce":
        nin, n, root, seg = int(parts[4][1:]), int(parts[5][1:]), int(parts[6][1:]), int(parts[7][1:])
        nout = 1
    else:
        nin, nout, n, seg = int(parts[4][1:]), int(parts[5][1:]), int(parts[6][1:]), int(parts[7][1:])
        root = 0
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "meta.txt"), "w").write(f"{kind} {op} {dtype} {P} {nin} {nout} {n} {root} {seg}\n")
        init.tofile(os.path.join(d, "init.bin"))
        if nin:
            z[case + "/in"].tofile(os.path.join(d, "in.bin"))
        r = subprocess.run([t.PROGRAM, d, mode], capture_output=True, text=True, timeout=timeout)
        if r.returncode != 0:
            return "FAIL rc %d: %s %s" % (r.returncode, r.stdout[-600:], r.stderr[-600:])
        bad = []
        for rank in range(P):
            if kind == "reduce" and rank != root and mode == "device":
                continue
            for call in range(2):
                got = np.fromfile(os.path.join(d, f"out_{rank}_{call}.bin"), dtype=init.dtype).reshape(nout, n)
                expect = want[rank] if kind == "reduce" else want
                for j in range(nout):
                    if got[j].view(np.uint8).tobytes() != expect.view(np.uint8).tobytes():
                        k = np.nonzero(got[j].view(np.uint8) != expect.view(np.uint8))[0]
                        bad.append((rank, call, j, int(k[0]) // init.itemsize, got[j][k[0] // init.itemsize],
                                    expect[k[0] // init.itemsize], len(k)))
        return "ok" if not bad else "MISMATCH %s" % bad[:4]


if __name__ == "__main__":
    mode = sys.argv[1]
    subs = sys.argv[2:]
    for src, case in t._cases():
        if subs and not any(s in case for s in subs):
            continue
        print(mode, case, run(src, case, mode), flush=True)
