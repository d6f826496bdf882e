"""GPU: the sliced interpreter's slice cap follows co-residency.

A sliced launch's workgroups spin until their peer slices run, so every
launch of the ranks sharing one GPU must be resident at once.  Round 5
measured 4 rank processes x 128 slices on one MI355X timing out in every
rank's device wait.  The executor now caps a rank's slices at the GPU's CU
count divided by the ranks on that GPU (executor_modes.cc coResidentSlices):
with GLOO_AMD_INTERP_MAX_SLICES=128 and 4 ranks on the one GPU, 256 / 4 = 64
slices, and the runs are exact.  The mesh halving-doubling plan at 4 Mi fp32
per rank has 4 MiB messages: 128 slices of 32 KiB wanted, 64 of 64 KiB run.
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
import json, os, sys
sys.path.insert(0, os.environ["GLOO_AMD_ROOT"])
sys.path.insert(0, os.path.join(os.environ["GLOO_AMD_ROOT"], "tests"))
import numpy as np
import gloo_amd, hip_rt
rank, P, store = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
hip_rt.set_device(0)
ctx = gloo_amd.Context(rank, P, store, device=0, timeout_ms=30000)
n = 4 << 20
buf = hip_rt.malloc(4 * n)
a = gloo_amd.Algorithm(ctx, "halving_doubling", "sum", "f32", [buf], n)
x = (np.arange(n, dtype=np.int64) % 1000).astype(np.float32)
res = []
for it in range(3):
    hip_rt.h2d(buf, x * (rank + 1 + it))
    a.run()
    y = hip_rt.d2h(buf, np.empty(n, np.float32))
    want = x * sum(r + 1 + it for r in range(P))
    res.append({"ok": bool((y == want).all()), "slices": a.mode()["interp_slices"]})
a.close()
ctx.close()
print("RESULT" + json.dumps(res), flush=True)
'''


@pytest.mark.timeout(240)
def test_slice_cap_four_ranks_one_gpu():
    P = 4
    torch = pytest.importorskip("torch")
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    with tempfile.TemporaryDirectory() as d:
        w = os.path.join(d, "w.py")
        open(w, "w").write(WORKER)
        e = dict(os.environ, GLOO_AMD_ROOT=ROOT, GLOO_AMD_INTERP_MAX_SLICES="128")
        procs = [subprocess.Popen([sys.executable, w, str(r), str(P), "file:" + os.path.join(d, "s")], env=e,
                                  stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(P)]
        outs = []
        try:
            for p in procs:
                outs.append(p.communicate(timeout=200))
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
    assert [p.returncode for p in procs] == [0] * P, "\n".join(e[-2500:] for _, e in outs)
    want_slices = min(128, cus // P)
    for r, (o, _) in enumerate(outs):
        for it, x in enumerate(json.loads(o.split("RESULT", 1)[1])):
            assert x["ok"], (r, it, x)
            assert x["slices"] == want_slices, (r, it, x, cus)
