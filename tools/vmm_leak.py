#!/usr/bin/env python3
"""Device memory of the cross-process pool as executors come and go.  Two
rank processes (no torch) build an HD executor of a new size every
iteration, run it and close it; rank 0 prints the device's used bytes
(hipMemGetInfo: both ranks share the GPU) and the pool's stats per
iteration.  The round-5 runs (profiles/round5/r5i_*) also trimmed the pool
collectively after each close, through the gloo_hip_ipc_trim of that
round's two-mechanism pool (since removed): VMM memory came back only when
its virtual range was freed, which is why the pool now never frees a slab.
usage: vmm_leak.py ITERS [ENV=VAL ...]"""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = r'''
import json, os, sys
import numpy as np
sys.path.insert(0, os.environ["GLOO_AMD_ROOT"]); sys.path.insert(0, os.path.join(os.environ["GLOO_AMD_ROOT"], "tests"))
import gloo_amd, hip_rt
rank, store, iters = int(sys.argv[1]), sys.argv[2], int(sys.argv[3])
hip_rt.set_device(0)
ctx = gloo_amd.Context(rank, 2, store, device=0, timeout_ms=30000)
free0, total = hip_rt.mem_info()
n = 1 << 22
buf = hip_rt.malloc(4 * n)
for it in range(iters):
    m = (1 << 18) * (1 + it % 16)
    x = np.full(m, rank + 1, np.float32)
    hip_rt.h2d(buf, x)
    a = gloo_amd.Algorithm(ctx, "halving_doubling", "sum", "f32", [buf], m)
    a.run()
    ok = bool((hip_rt.d2h(buf, x) == 3).all())
    a.close()
    st = gloo_amd.ipc_stats()
    if rank == 0:
        print(json.dumps({"it": it, "elems": m, "ok": ok, "used_mb": round((free0 - hip_rt.mem_info()[0]) / 2**20, 1),
                          "slabs": st["slabs"], "slab_bytes": st["slab_bytes"], "mapped": st["peer_slabs_mapped"]}), flush=True)
ctx.close()
'''


def main():
    iters = int(sys.argv[1])
    env = dict(os.environ, GLOO_AMD_ROOT=ROOT)
    for kv in sys.argv[2:]:
        k, v = kv.split("=", 1)
        env[k] = v
    with tempfile.TemporaryDirectory() as d:
        w = os.path.join(d, "w.py")
        open(w, "w").write(WORKER)
        procs = [subprocess.Popen([sys.executable, w, str(r), "file:" + os.path.join(d, "s"), str(iters)], env=env,
                                  stdout=None if r == 0 else subprocess.DEVNULL) for r in range(2)]
        rcs = [p.wait(timeout=300) for p in procs]
    print(json.dumps({"rcs": rcs}))
    return 0 if rcs == [0, 0] else 1


if __name__ == "__main__":
    sys.exit(main())
