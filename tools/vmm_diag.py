#!/usr/bin/env python3
"""Diagnosis of the VMM cross-process pool: P rank processes run one
allreduce (HD or ring-chunked) of N fp32 twice with a short context timeout,
GLOO_AMD_TRACE=1; each rank's stdout/stderr goes to gpurun_out/vmmdiag_<label>_r<rank>.log.
usage: vmm_diag.py LABEL ALGO P N [ENV=VAL ...]"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = r'''
import os, sys, time, faulthandler
faulthandler.enable()
import numpy as np
sys.path.insert(0, os.environ["GLOO_AMD_ROOT"]); sys.path.insert(0, os.path.join(os.environ["GLOO_AMD_ROOT"], "tests"))
import gloo_amd, hip_rt
rank, size, store, algo, n = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], int(sys.argv[5])
hip_rt.set_device(0)
x = np.full(n, rank + 1, np.float32)
buf = hip_rt.malloc(x.nbytes)
hip_rt.h2d(buf, x)
ctx = gloo_amd.Context(rank, size, store, device=0, timeout_ms=15000)
t0 = time.time()
a = gloo_amd.Algorithm(ctx, algo, "sum", "f32", [buf], n)
print("constructed", round(time.time() - t0, 3), a.mode(), flush=True)
for it in range(3):
    hip_rt.h2d(buf, x)
    a.run()
    y = hip_rt.d2h(buf, x)
    print("run", it, "ok" if (y == size * (size + 1) / 2).all() else "BAD %s" % y[:4], flush=True)
a.close(); ctx.close()
print("closed", flush=True)
'''


def main():
    label, algo, P, n = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    env = dict(os.environ, GLOO_AMD_ROOT=ROOT, GLOO_AMD_TRACE="1")
    for kv in sys.argv[5:]:
        k, v = kv.split("=", 1)
        env[k] = v
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with tempfile.TemporaryDirectory() as d:
        w = os.path.join(d, "w.py")
        open(w, "w").write(WORKER)
        logs = [open(os.path.join(ROOT, "gpurun_out", f"vmmdiag_{label}_r{r}.log"), "w") for r in range(P)]
        procs = [subprocess.Popen([sys.executable, w, str(r), str(P), "file:" + os.path.join(d, "s"), algo, str(n)],
                                  env=env, stdout=logs[r], stderr=subprocess.STDOUT) for r in range(P)]
        rcs = []
        for p in procs:
            try:
                rcs.append(p.wait(timeout=60))
            except subprocess.TimeoutExpired:
                p.kill()
                rcs.append("timeout")
        print(label, rcs, flush=True)
        return 0 if all(r == 0 for r in rcs) else 1


if __name__ == "__main__":
    sys.exit(main())
