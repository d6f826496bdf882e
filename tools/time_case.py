#!/usr/bin/env python3
"""Where the seconds of one multi-process golden case go (developer tool).

Launches P rank processes of one tests/golden/sched_golden.npz case on GPU 0,
the way tests/test_collectives_gpu.py does, with GLOO_AMD_TRACE=1, and prints
every rank's stderr line and phase mark prefixed by seconds since launch.
  python tools/time_case.py reduce_scatter/max/bf16/P8/n4096 [VAR=VAL ...]
"""
import os
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import os, sys, time
t0 = float(os.environ["T0"])
def mark(what):
    print("PHASE %.3f %s" % (time.time() - t0, what), file=sys.stderr, flush=True)
mark("python up")
import numpy as np
sys.path.insert(0, os.environ["GLOO_AMD_ROOT"])
import torch, gloo_amd
mark("imports done")
rank, size, store, case = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
g = np.load(os.path.join(os.environ["GLOO_AMD_ROOT"], "tests", "golden", "sched_golden.npz"))
algo, op, dtype = case.split("/")[:3]
x = g[case + "/in"]
recv = g[case + "/recv"] if algo == "reduce_scatter" else None
xr = x[rank] if algo == "reduce_scatter" else x[rank, 0]
torch.cuda.set_device(0)
buf = torch.from_numpy(xr.view(np.uint8).copy()).to("cuda:0")
torch.cuda.synchronize()
mark("buffer on GPU")
ctx = gloo_amd.Context(rank, size, store, device=0, timeout_ms=60000)
mark("context")
a = gloo_amd.Algorithm(ctx, algo, op, dtype, [buf.data_ptr()], xr.size, recv_elems=recv)
mark("algorithm")
a.run()
mark("run 1")
a.run()
mark("run 2")
a.close()
mark("algorithm closed")
ctx.close()
mark("context closed")
'''


def main():
    case = sys.argv[1]
    extra = dict(kv.split("=", 1) for kv in sys.argv[2:])
    P = int(case.split("/")[3][1:])
    t0 = time.time()
    with tempfile.TemporaryDirectory() as d:
        w = os.path.join(d, "w.py")
        open(w, "w").write(WORKER)
        env = dict(os.environ, GLOO_AMD_ROOT=ROOT, GLOO_AMD_TRACE="1", T0=repr(t0), **extra)
        procs = [subprocess.Popen([sys.executable, "-u", w, str(r), str(P), "file:" + os.path.join(d, "s"), case],
                                  env=env, stderr=subprocess.PIPE, text=True) for r in range(P)]

        def pump(r, p):
            for line in p.stderr:
                print("%8.3f r%d %s" % (time.time() - t0, r, line.rstrip()), flush=True)
        ts = [threading.Thread(target=pump, args=(r, p)) for r, p in enumerate(procs)]
        for t in ts:
            t.start()
        rcs = [p.wait(timeout=300) for p in procs]
        for t in ts:
            t.join()
    print("exit codes", rcs, "total %.3f s" % (time.time() - t0))
    sys.exit(0 if rcs == [0] * P else 1)


if __name__ == "__main__":
    main()
