"""GPU: algorithms given no stream each run on their own.

Round 5 had every algorithm of a context that was given no stream share one
stream of the context.  Two algorithms of one context run from two threads,
started in opposite orders on the two ranks, then queued each one's
device-side waits behind the other's kernels: rank 0's stream held
[A waits for rank 1's A][B], rank 1's [B waits for rank 0's B][A] — a
deadlock until the timeout.  The reference gives each op its own stream
(gloo/cuda.h:102-105, gloo/cuda_allreduce_ring_chunked.cc:55-67); so does
the executor now.  Ranks are processes (device-side signalling), each
running its two algorithms concurrently from two threads, three times.
"""
import json
import os
import subprocess
import sys
import tempfile

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import json, os, sys, threading, time
sys.path.insert(0, os.environ["GLOO_AMD_ROOT"])
sys.path.insert(0, os.path.join(os.environ["GLOO_AMD_ROOT"], "tests"))
import numpy as np
import gloo_amd, hip_rt
rank, store, algo = int(sys.argv[1]), sys.argv[2], sys.argv[3]
hip_rt.set_device(0)
ctx = gloo_amd.Context(rank, 2, store, device=0, timeout_ms=20000)
n = 1 << 16
bufs = [hip_rt.malloc(4 * n) for _ in range(2)]
# constructed in the same order on both ranks (construction is collective)
algos = [gloo_amd.Algorithm(ctx, algo, "sum", "f32", [bufs[k]], n) for k in range(2)]
res = []
for it in range(3):
    for k in range(2):
        hip_rt.h2d(bufs[k], np.full(n, (rank + 1) * (k + 1) * (it + 1), np.float32))
    errs = []

    def go(k):
        try:
            algos[k].run()
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    order = [0, 1] if (rank + it) % 2 == 0 else [1, 0]
    ts = []
    for k in order:
        t = threading.Thread(target=go, args=(k,))
        t.start()
        ts.append(t)
        time.sleep(0.05)
    for t in ts:
        t.join()
    hip_rt.synchronize()
    vals = [hip_rt.d2h(b, np.empty(n, np.float32)) for b in bufs]
    res.append({"errs": errs, "ok": [bool((vals[k] == 3 * (k + 1) * (it + 1)).all()) for k in range(2)]})
for a in algos:
    a.close()
ctx.close()
print("RESULT" + json.dumps(res), flush=True)
'''


@pytest.mark.timeout(240)
@pytest.mark.parametrize("algo", ["halving_doubling", "ring_chunked"])
def test_two_threads_opposite_orders(algo):
    with tempfile.TemporaryDirectory() as d:
        w = os.path.join(d, "w.py")
        open(w, "w").write(WORKER)
        e = dict(os.environ, GLOO_AMD_ROOT=ROOT)
        procs = [subprocess.Popen([sys.executable, w, str(r), "file:" + os.path.join(d, "s"), algo], env=e,
                                  stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
        outs = []
        try:
            for p in procs:
                outs.append(p.communicate(timeout=200))
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
    assert [p.returncode for p in procs] == [0, 0], "\n".join(e[-2500:] for _, e in outs)
    for r, (o, _) in enumerate(outs):
        for it, x in enumerate(json.loads(o.split("RESULT", 1)[1])):
            assert not x["errs"] and all(x["ok"]), (r, it, x)
