"""GPU: the IPC slab pool stays bounded (ipc.h).

Two rank processes build halving-doubling executors (mesh route: their inbox
arenas are exported slabs) of ten size classes in sequence, then walk back
down through classes that a trim freed.  With GLOO_AMD_IPC_POOL_MAX = 256 MiB
the pool never holds more than the ceiling beyond the slabs of the live
executor (an executor's construction trims collectively first), trims
happen, their addresses are retired (never exported again for other pages),
every run is exact (the closed form of rank r contributing (7 i + r) mod
4096 at element i), and an explicit collective gloo_hip_ipc_trim leaves no
slab and no mapping."""
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
import torch, gloo_amd
rank, store = int(sys.argv[1]), sys.argv[2]
torch.cuda.set_device(0)
ctx = gloo_amd.Context(rank, 2, store, device=0, timeout_ms=60000)
sizes = [1 << k for k in range(19, 29)] + [1 << 27, 1 << 21, 1 << 24, 3 << 22]
out = []
for n in sizes:
    i7 = torch.arange(n, device="cuda:0", dtype=torch.int64) * 7
    buf = ((i7 + rank) % 4096).float()
    want = ((i7 % 4096) + ((i7 + 1) % 4096)).float()
    del i7
    a = gloo_amd.Algorithm(ctx, "halving_doubling", "sum", "f32", [buf.data_ptr()], n)
    st = gloo_amd.ipc_stats()
    ok = []
    for it in range(2):
        if it:
            buf.copy_(((torch.arange(n, device="cuda:0", dtype=torch.int64) * 7 + rank) % 4096).float())
            torch.cuda.synchronize()  # the executor runs on its own stream
        a.run()
        torch.cuda.synchronize()
        ok.append(bool((buf == want).all()))
    a.close()
    out.append({"n": n, "ok": ok, "stats": st})
    del buf, want
final = gloo_amd.ipc_stats()
gloo_amd.ipc_trim(ctx)   # collective: every unused slab and mapping goes
trimmed = gloo_amd.ipc_stats()
ctx.close()
print("RESULT" + json.dumps({"steps": out, "final": final, "trimmed": trimmed}), flush=True)
'''


@pytest.mark.timeout(300)
def test_ipc_pool_bounded_with_trims():
    pytest.importorskip("torch")
    cap = 256 << 20
    with tempfile.TemporaryDirectory() as d:
        w = os.path.join(d, "w.py")
        open(w, "w").write(WORKER)
        e = dict(os.environ, GLOO_AMD_ROOT=ROOT, GLOO_AMD_IPC_POOL_MAX=str(cap), GLOO_AMD_TRACE="1")
        procs = [subprocess.Popen([sys.executable, w, str(r), "file:" + os.path.join(d, "s")], env=e,
                                  stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
        outs = []
        try:
            for p in procs:
                outs.append(p.communicate(timeout=280))
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        assert [p.returncode for p in procs] == [0, 0], "\n".join(f"rank {r}: {e[-2500:]}"
                                                              for r, (o, e) in enumerate(outs))
        res = [json.loads(o.split("RESULT", 1)[1]) for o, e in outs]
    for r in res:
        for s in r["steps"]:
            assert s["ok"] == [True, True], s
            live = 4 * s["n"] + (8 << 20)  # this executor's arena (about n fp32) and mailbox, rounded up
            assert s["stats"]["slab_bytes"] <= cap + 2 * live, s
            assert s["stats"]["pool_max_bytes"] == cap
        f = r["final"]
        assert f["trims"] >= 1 and f["retired_addresses"] >= 1, f
        assert f["slab_bytes"] <= cap + 4 * r["steps"][-1]["n"] + (8 << 20), f
        t = r["trimmed"]
        assert t["slabs"] == 0 and t["slab_bytes"] == 0 and t["free"] == 0, t
        assert t["peer_slabs_mapped"] == 0, t
