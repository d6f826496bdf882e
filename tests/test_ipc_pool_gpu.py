"""GPU: the cross-process slab pool stays bounded (ipc.h).

The pool's slabs are HIP VMM blocks that are never freed while the process
lives (a freed virtual range handed out again shows stale pages) and are
reused by size class instead.  test_ipc_pool_reuses_size_classes: two rank
processes build halving-doubling executors (mesh route: their inbox arenas
are exported slabs) of ten size classes in sequence, then walk back down
through classes already used: the walk back creates no slab and maps no new
peer slab, every slab is back in the free list after its executor closes,
and every run is exact (the closed form of rank r contributing (7 i + r)
mod 4096 at element i)."""
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
sizes = json.loads(os.environ.get("GLOO_AMD_TEST_SIZES", "null")) or \
    [1 << k for k in range(19, 29)] + [1 << 27, 1 << 21, 1 << 24, 3 << 22]
out = []
for n in sizes:
    i7 = torch.arange(n, device="cuda:0", dtype=torch.int64) * 7
    buf = ((i7 + rank) % 4096).float()
    want = ((i7 % 4096) + ((i7 + 1) % 4096)).float()
    del i7
    a = gloo_amd.Algorithm(ctx, "halving_doubling", "sum", "f32", [buf.data_ptr()], n)
    ok = []
    for it in range(2):
        if it:
            buf.copy_(((torch.arange(n, device="cuda:0", dtype=torch.int64) * 7 + rank) % 4096).float())
            torch.cuda.synchronize()  # the executor runs on its own stream
        a.run()
        torch.cuda.synchronize()
        ok.append(bool((buf == want).all()))
    a.close()
    out.append({"n": n, "ok": ok, "stats": gloo_amd.ipc_stats()})
    del buf, want
ctx.close()
print("RESULT" + json.dumps({"steps": out}), flush=True)
'''


def run_pair(worker, args, env, timeout):
    with tempfile.TemporaryDirectory() as d:
        w = os.path.join(d, "w.py")
        open(w, "w").write(worker)
        e = dict(os.environ, GLOO_AMD_ROOT=ROOT, **env)
        procs = [subprocess.Popen([sys.executable, w, str(r), "file:" + os.path.join(d, "s")] + args, env=e,
                                  stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
        outs = []
        try:
            for p in procs:
                outs.append(p.communicate(timeout=timeout))
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        assert [p.returncode for p in procs] == [0, 0], "\n".join(f"rank {r}: {e[-2500:]}"
                                                              for r, (o, e) in enumerate(outs))
        return [json.loads(o.split("RESULT", 1)[1]) for o, e in outs]


@pytest.mark.timeout(300)
def test_ipc_pool_reuses_size_classes():
    pytest.importorskip("torch")
    res = run_pair(WORKER, [], {}, 280)
    for r in res:
        steps = r["steps"]
        for s in steps:
            assert s["ok"] == [True, True], s
            st = s["stats"]
            assert st["free"] == st["slabs"], s   # every slab back in the pool
        up, down = steps[9]["stats"], steps[-1]["stats"]
        # the walk back down reuses: no new slab, no new peer mapping
        assert down["slabs"] == up["slabs"] and down["slab_bytes"] == up["slab_bytes"], (up, down)
        assert down["peer_slabs_mapped"] == up["peer_slabs_mapped"] and down["imports"] == up["imports"], (up, down)
        # ten arena classes (2 MiB .. 1 GiB, an arena of n fp32 rounds up to
        # at most 2 x 4 n B) and the mailboxes' class: below 2 x the sum
        assert up["slab_bytes"] <= 2 * sum(4 * s["n"] for s in steps[:10]) + (64 << 20), up


@pytest.mark.timeout(200)
def test_ipc_pool_best_fit_decreasing_sizes():
    """a request of a class never used before is served from a
    larger idle slab (best fit) instead of a new one.  Halving-doubling
    executors of strictly decreasing size classes, each closed before the
    next: the first creates the arena slab (and the mailbox's), no later one
    creates any, and every run is exact."""
    pytest.importorskip("torch")
    sizes = [1 << 25, 3 << 22, 1 << 23, 1 << 22, 1 << 21, 1 << 20]
    res = run_pair(WORKER, [], {"GLOO_AMD_TEST_SIZES": json.dumps(sizes)}, 180)
    for r in res:
        steps = r["steps"]
        for s in steps:
            assert s["ok"] == [True, True], s
        first = steps[0]["stats"]
        for s in steps[1:]:
            assert s["stats"]["slabs"] == first["slabs"], (first, s)
            assert s["stats"]["slab_bytes"] == first["slab_bytes"], (first, s)


CHURN_WORKER = r'''
import json, os, random, sys
import numpy as np
sys.path.insert(0, os.environ["GLOO_AMD_ROOT"])
sys.path.insert(0, os.path.join(os.environ["GLOO_AMD_ROOT"], "tests"))
import gloo_amd, hip_rt
rank, store, count = int(sys.argv[1]), sys.argv[2], int(sys.argv[3])
hip_rt.set_device(0)
free0 = hip_rt.mem_info()[0]
ctx = gloo_amd.Context(rank, 2, store, device=0, timeout_ms=60000)
rng = random.Random(5)   # the same sequence on both ranks
algos = ["halving_doubling", "ring_chunked", "reduce_scatter"]
bad, peak_used = [], 0
for it in range(count):
    n = 1 << rng.randrange(12, 23)
    n += rng.randrange(0, 4096)
    algo = algos[rng.randrange(len(algos))]
    i = np.arange(n, dtype=np.int64)
    x = ((7 * i + rank) % 4096).astype(np.float32)
    want = (((7 * i) % 4096) + ((7 * i + 1) % 4096)).astype(np.float32)
    buf = hip_rt.malloc(x.nbytes)
    hip_rt.h2d(buf, x)
    recv = [n // 2 + (n % 2), n // 2] if algo == "reduce_scatter" else None
    a = gloo_amd.Algorithm(ctx, algo, "sum", "f32", [buf], n, recv_elems=recv)
    a.run()
    y = hip_rt.d2h(buf, x)
    m = recv[rank] if recv else n
    if recv:   # reduce-scatter: rank r's block sits at the start of its buffer
        off = 0 if rank == 0 else recv[0]
        ok = bool((y[:m] == want[off:off + m]).all())
    else:
        ok = bool((y == want).all())
    if not ok:
        bad.append((it, algo, n))
    a.close()
    hip_rt.free(buf)
    peak_used = max(peak_used, free0 - hip_rt.mem_info()[0])
st = gloo_amd.ipc_stats()
ctx.close()
print("RESULT" + json.dumps({"bad": bad, "stats": st, "peak_used": peak_used,
                             "end_used": free0 - hip_rt.mem_info()[0]}), flush=True)
'''


@pytest.mark.timeout(400)
def test_ipc_pool_churn_bounded():
    """VERDICT r4 "next round" 2: pool churn.  200 executor constructions of
    random size classes (arenas of 16 KiB to 32 MiB) and algorithms stay
    exact and bounded.  The rounds 3-4 hipIpc pool under a 64 MiB ceiling
    failed exactly this (a collective trim before almost every construction;
    "no exportable block ... after 64 tries (retired ranges)",
    profiles/round5/r5c_pytest_churn_hipipc.log).  The VMM pool never frees
    a slab and reuses them by size class instead, so it holds at most one
    slab per class and kind per live executor: here below 256 MiB per
    rank."""
    pytest.importorskip("torch")
    res = run_pair(CHURN_WORKER, ["200"], {}, 380)
    for r in res:
        assert r["bad"] == [], r["bad"]
        st = r["stats"]
        assert st["free"] == st["slabs"], st
        # classes 2 MiB .. 64 MiB (2 x the largest arena, rounded up), arena and
        # mailbox kinds: 2 x 126 MiB at most
        assert st["slab_bytes"] <= 256 << 20, st
        # both ranks' pools and user buffers (16 MiB) share this one GPU, plus
        # runtime slack
        assert r["peak_used"] <= 2 * (256 << 20) + 2 * (16 << 20) + (512 << 20), r
