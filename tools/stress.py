#!/usr/bin/env python3
"""Mixed-collective stress run (developer tool): P rank processes on one GPU
each build the same set of algorithms — ring-chunked, halving-doubling, ring,
reduce-scatter; sum / max / min over f32 / bf16 / i32; sizes from 1 element to
8 MiB, so every launch mode (fused steps, interpreter one- and many-workgroup,
graph replay, eager) appears; plus new-style gloo::allreduce RING / BCUBE and
gloo::reduce calls with separate input and output — and then run them in one shared seeded random
order for `seconds`, refilling inputs and checking every result exactly
against its closed form (rank r contributes r + 1 at every position, or
(r + 1) * (i % 7 + 1) for sum).  A wrong byte, a timeout or a fault ends the
run with a non-zero exit.  One JSON line per rank at the end.

  python tools/stress.py <ranks> <seconds> [seed]
STRESS_BIG=1 adds 16 MiB and 64 MiB cases (eager and graph-replayed mesh plans).
"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import json, os, sys, time


def emit(o):
    # one write per line: the ranks share the parent's stdout, and print()'s
    # separate newline write let two ranks' lines run together
    os.write(1, (json.dumps(o) + "\n").encode())


import numpy as np
sys.path.insert(0, os.environ["GLOO_AMD_ROOT"])
import torch, gloo_amd
rank, P, store, seconds, seed = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], float(sys.argv[4]), int(sys.argv[5])
torch.cuda.set_device(0)
dev = torch.device("cuda:0")
ctx = gloo_amd.Context(rank, P, store, device=0, timeout_ms=60000)
tdt = {"f32": torch.float32, "bf16": torch.bfloat16, "i32": torch.int32}
cases = []
sizes = [1, 7, 1000, 4099, 65536 + 3, (1 << 20) + 5, 2 << 20]
if os.environ.get("STRESS_BIG") == "1":  # the eager and graph launch modes of the mesh routes (>= 4 MiB messages)
    sizes += [(4 << 20) + 3, 16 << 20]
combos = (("sum", "f32"), ("max", "bf16"), ("min", "i32"), ("sum", "i32"))
# a context holds at most 64 live algorithms: one op / dtype per (schedule, size), rotating
# (AllreduceBcube sums every rank only where P is a power of its base, 2 here)
schedules = ("ring_chunked", "halving_doubling", "ring", "reduce_scatter") + (("bcube",) if P & (P - 1) == 0 else ())
for ai, algo in enumerate(schedules):
    for si, n in enumerate(sizes):
        if algo == "ring" and n > (1 << 20):  # (the plain ring moves the whole buffer per hop)
            continue
        op, dt = combos[(ai + si) % len(combos)]
        cases.append((algo, op, dt, n))
built = []
for algo, op, dt, n in cases:
    buf = torch.zeros(n, dtype=tdt[dt], device=dev)
    recv = None
    if algo == "reduce_scatter":
        chunk = (n + P - 1) // P
        recv, rem = [], n
        for _ in range(P):
            recv.append(min(chunk, rem))
            rem = rem - chunk if rem > chunk else 0
    a = gloo_amd.Algorithm(ctx, algo, op, dt, [buf.data_ptr()], n, recv_elems=recv,
                           base=2 if algo == "bcube" else None)
    idx = torch.arange(n, device=dev)
    if op == "sum":
        mine = ((rank + 1) * (idx % 7 + 1)).to(tdt[dt])
        want = (P * (P + 1) // 2 * (idx % 7 + 1)).to(tdt[dt])
    else:
        mine = torch.full((n,), rank + 1, dtype=tdt[dt], device=dev)
        want = torch.full((n,), P if op == "max" else 1, dtype=tdt[dt], device=dev)
    if recv is not None:  # rank r's block (global offset sum(recv[:r])) lands at the front
        off = sum(recv[:rank])
        want = want[off:off + recv[rank]]
    lim = recv[rank] if recv is not None else n
    built.append((a, buf, mine, want, lim, (algo, op, dt, n)))
# new-style calls (gloo::allreduce RING / BCUBE, gloo::reduce to a rotating
# root) with separate input and output: out = sum over ranks of in
class NewStyle:
    def __init__(self, kind, n, root=0):
        self.kind, self.n, self.root = kind, n, root
        self.inp = torch.zeros(n, dtype=torch.float32, device=dev)
        self.out = torch.zeros(n, dtype=torch.float32, device=dev)
    def run(self):
        if self.kind == "reduce":
            gloo_amd.reduce_to_root(ctx, self.out.data_ptr(), self.n, "f32", self.root, "sum", input=self.inp.data_ptr())
        else:
            gloo_amd.allreduce(ctx, [self.out.data_ptr()], self.n, "f32", "sum", inputs=[self.inp.data_ptr()],
                               algorithm=self.kind)
    def mode(self):
        return {"interp": False, "graph": False}
for kind in ("ring", "bcube", "reduce"):
    for j, n in enumerate((1000, 65539, (1 << 20) + 5)):
        ns = NewStyle(kind, n, root=j % P)
        idx = torch.arange(n, device=dev)
        mine = ((rank + 1) * (idx % 7 + 1)).to(torch.float32)
        want = (P * (P + 1) // 2 * (idx % 7 + 1)).to(torch.float32)
        # the reduce's non-root outputs are unspecified: check the root only
        lim = n if (kind != "reduce" or rank == ns.root) else 0
        built.append((ns, ns.out, mine, want[:lim], lim, ("new_" + kind, "sum", "f32", n)))
        ns.inp.copy_(mine)
flag = torch.zeros(1, dtype=torch.int32, device=dev)
stopper = gloo_amd.Algorithm(ctx, "ring_chunked", "max", "i32", [flag.data_ptr()], 1)
order = np.random.default_rng(seed + 1)
t0 = time.time()
runs = 0
modes = {}
while True:
    # every rank draws the same case; a run ends only on a round boundary all agree on
    k = int(order.integers(len(built)))
    a, buf, mine, want, lim, key = built[k]
    if key[0].startswith("new_"):
        buf.zero_()  # the output; the input keeps this rank's contribution
    else:
        buf.copy_(mine)
    torch.cuda.synchronize()
    a.run()
    torch.cuda.synchronize()
    if not bool((buf[:lim] == want).all()):
        bad = int((buf[:lim] != want).sum())
        emit({"rank": rank, "error": "wrong result", "case": key, "bad": bad, "runs": runs})
        sys.exit(2)
    runs += 1
    m = a.mode()
    label = key[0] + "/" + ("call" if isinstance(a, NewStyle) else
                            "interp" if m["interp"] else "graph" if m["graph"] else "eager")
    modes[label] = modes.get(label, 0) + 1
    if runs % 200 == 0:
        # agree on stopping: rank 0's clock decides, through a one-element max allreduce
        flag.fill_(1 if (rank == 0 and time.time() - t0 > seconds) else 0)
        torch.cuda.synchronize()
        stopper.run()
        torch.cuda.synchronize()
        if int(flag.item()):
            break
for a, *_ in built:
    if not isinstance(a, NewStyle):
        a.close()
stopper.close()
ctx.close()
emit({"rank": rank, "runs": runs, "seconds": round(time.time() - t0, 1), "cases": len(built),
                  "modes": modes})
'''


def main():
    P = int(sys.argv[1])
    seconds = float(sys.argv[2])
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    with tempfile.TemporaryDirectory() as d:
        w = os.path.join(d, "w.py")
        open(w, "w").write(WORKER)
        env = dict(os.environ, GLOO_AMD_ROOT=ROOT)
        procs = [subprocess.Popen([sys.executable, "-u", w, str(r), str(P), "file:" + os.path.join(d, "s"),
                                   str(seconds), str(seed)], env=env) for r in range(P)]
        rcs = [p.wait(timeout=seconds + 600) for p in procs]
    print(json.dumps({"ranks": P, "exit_codes": rcs}), flush=True)
    sys.exit(0 if rcs == [0] * P else 1)


if __name__ == "__main__":
    main()
