"""GPU: gloo::allreduce(opts) with BCUBE and gloo::reduce(opts) through the
C-ABI (gloo_hip_allreduce / gloo_hip_reduce_to_root), against the reference's
own outputs (tests/golden/newstyle_golden.npz, oracle/gen_golden.py).

Ranks as threads of one process (host-signalled, the pattern of
gloo/test/base_test.h:107-152) and as processes (device-signalled, inboxes
over HIP IPC, hipGraph replay of the cached schedule).
"""
import json
import os
import subprocess
import sys
import tempfile
import threading
import uuid

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "newstyle_golden.npz")


@pytest.fixture(scope="module")
def torch():
    t = pytest.importorskip("torch")
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.fixture(scope="module")
def golden_new():
    return np.load(GOLDEN)


def _keys(prefix, max_p=8):
    z = np.load(GOLDEN)
    keys = sorted({k.rsplit("/", 1)[0] for k in z.files if k.startswith(prefix)})
    return [k for k in keys if int(k.split("/")[3][1:]) <= max_p]


def same_bytes(a, b):
    return a.shape == b.shape and (a.view(np.uint8) == b.view(np.uint8)).all()


def run_threads(P, body):
    errors = []
    ts = [threading.Thread(target=lambda r=r: _guard(body, r, errors)) for r in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


def _guard(body, r, errors):
    try:
        body(r)
    except Exception as e:  # noqa: BLE001
        errors.append((r, repr(e)))


def _bcube_cases():
    """Every bcube golden: both routes up to P = 8 (the mesh plan's range),
    the reference's route alone above (P = 12: 3 x 4 groups)."""
    out = []
    for k in _keys("bcube/", max_p=64):
        for mesh in (["1", "0"] if int(k.split("/")[3][1:]) <= 8 else ["0"]):
            out.append((k, mesh))
    return out


@pytest.mark.parametrize("case,mesh", _bcube_cases())
def test_bcube_threads_golden(torch, golden_new, case, mesh, monkeypatch):
    """BCUBE allreduce, ranks as threads on the visible GPU(s); called twice
    (the second call reuses the cached schedule with rebound buffers).  Both
    routes: the derived mesh plan (default, 2 <= P <= 8) and the reference's."""
    import gloo_amd
    monkeypatch.setenv("GLOO_AMD_MESH", mesh)
    parts = case.split("/")
    op, dtype, P = parts[1], parts[2], int(parts[3][1:])
    nin, nout, n = int(parts[4][1:]), int(parts[5][1:]), int(parts[6][1:])
    init = golden_new[case + "/init"]
    ins = golden_new[case + "/in"] if nin else None
    want = golden_new[case + "/out"]
    url = "mem:" + uuid.uuid4().hex
    ngpu = torch.cuda.device_count()
    results = {}

    def body(r):
        d = torch.device("cuda", r % ngpu)
        torch.cuda.set_device(d)
        ctx = gloo_amd.Context(r, P, url, device=d.index, timeout_ms=60000)
        for rep in range(2):
            outs = [torch.from_numpy(init[r, j].view(np.uint8).copy()).to(d) for j in range(nout)]
            inb = [torch.from_numpy(ins[r, j].view(np.uint8).copy()).to(d) for j in range(nin)]
            torch.cuda.synchronize(d)
            gloo_amd.allreduce(ctx, [t.data_ptr() for t in outs], n, dtype, op,
                               inputs=[t.data_ptr() for t in inb], algorithm="bcube")
            results[(r, rep)] = [t.cpu().numpy().view(init.dtype) for t in outs]
            modes[(r, rep)] = ctx.last_mode()
        ctx.close()

    modes = {}
    run_threads(P, body)
    for (r, rep), outs in sorted(results.items()):
        for j, y in enumerate(outs):
            assert same_bytes(y, want), (r, rep, j, y, want)
    # every rank's inboxes are written by its peers' streams: fine-grained
    # (executor.cc; the cause of GPUTEST_r05's red case)
    assert all(m["fine_arena"] or m["host_arena"] for m in modes.values()), modes


@pytest.mark.parametrize("algo,P,mesh", [("bcube", 12, "0"), ("bcube", 4, "1"), ("ring", 3, "0")])
def test_threads_inboxes_fine_grained(torch, algo, P, mesh, monkeypatch):
    """GPUTEST_r05 (test_newstyle_plan.py::test_bcube_p12_stale_inbox_read_explains_r05):
    with ranks as threads on ONE GPU the inbox arena was coarse-grained, and
    the wrong value is what a second-run fold gives if it reads the first
    run's message at a shared offset (a stale line is the one cache path; it
    was not reproduced in isolation).  The fix, checked
    directly: every executor whose inboxes another rank writes reports a
    fine-grained arena, on the same-GPU thread route too; the results are
    exact over repeated calls with the buffers rebound each time."""
    import gloo_amd
    monkeypatch.setenv("GLOO_AMD_MESH", mesh)
    n = 4099
    url = "mem:" + uuid.uuid4().hex
    modes, bad = {}, []

    def body(r):
        torch.cuda.set_device(0)
        ctx = gloo_amd.Context(r, P, url, device=0, timeout_ms=60000)
        for rep in range(3):
            out = torch.full((n,), float(r + 1 + rep), device="cuda:0")
            torch.cuda.synchronize()
            gloo_amd.allreduce(ctx, [out.data_ptr()], n, "f32", "sum", algorithm=algo)
            want = P * (P + 1) / 2 + P * rep
            if not bool((out == want).all()):
                bad.append((r, rep))
            modes[(r, rep)] = ctx.last_mode()
        ctx.close()

    run_threads(P, body)
    assert not bad, bad
    assert all(m["fine_arena"] and not m["device_signal"] for m in modes.values()), modes


@pytest.mark.parametrize("mesh", ["1", "0"])
@pytest.mark.parametrize("case", _keys("reduce/"))
def test_reduce_threads_golden(torch, golden_new, case, mesh, monkeypatch):
    """gloo::reduce: the root's output equals the reference's on both routes;
    on the reference route every rank's whole output does (the others hold
    the partial sums the ring leaves; the mesh route leaves other scratch)."""
    import gloo_amd
    monkeypatch.setenv("GLOO_AMD_MESH", mesh)
    parts = case.split("/")
    op, dtype, P = parts[1], parts[2], int(parts[3][1:])
    has_in, n, root, seg = int(parts[4][1:]), int(parts[5][1:]), int(parts[6][1:]), int(parts[7][1:])
    init = golden_new[case + "/init"]
    ins = golden_new[case + "/in"] if has_in else None
    want = golden_new[case + "/out"]
    url = "mem:" + uuid.uuid4().hex
    ngpu = torch.cuda.device_count()
    results = {}

    def body(r):
        d = torch.device("cuda", r % ngpu)
        torch.cuda.set_device(d)
        ctx = gloo_amd.Context(r, P, url, device=d.index, timeout_ms=60000)
        for rep in range(2):
            out = torch.from_numpy(init[r, 0].view(np.uint8).copy()).to(d)
            inp = torch.from_numpy(ins[r, 0].view(np.uint8).copy()).to(d) if has_in else None
            torch.cuda.synchronize(d)
            gloo_amd.reduce_to_root(ctx, out.data_ptr(), n, dtype, root, op,
                                    input=inp.data_ptr() if inp is not None else None, max_segment_bytes=seg)
            results[(r, rep)] = out.cpu().numpy().view(init.dtype)
        ctx.close()

    run_threads(P, body)
    for (r, rep), y in results.items():
        if mesh == "0" or r == root:
            assert same_bytes(y, want[r]), (r, rep)


WORKER = r'''
import os, sys, json, numpy as np
sys.path.insert(0, os.environ["GLOO_AMD_ROOT"])
sys.path.insert(0, os.path.join(os.environ["GLOO_AMD_ROOT"], "tests"))
import gloo_amd, hip_rt
rank, size, store, kind, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], sys.argv[5]
n = int(os.environ.get("GLOO_AMD_TEST_N", "300000"))
hip_rt.set_device(0)
ctx = gloo_amd.Context(rank, size, store, device=0, timeout_ms=60000)
sets = [(hip_rt.malloc(4 * n), hip_rt.malloc(4 * n)) for _ in range(2)]
like = np.empty(n, np.float32)
res = []
modes = []
for it, s in enumerate([0, 0, 0, 1, 1, 0]):
    inp, outp = sets[s]
    hip_rt.h2d(inp, np.full(n, (rank + 1) * (it + 1), np.float32))
    hip_rt.h2d(outp, np.full(n, -1, np.float32))
    if kind in ("bcube", "ring"):
        gloo_amd.allreduce(ctx, [outp], n, "f32", "sum", inputs=[inp], algorithm=kind,
                           max_segment_bytes=128 << 10)
    else:
        gloo_amd.reduce_to_root(ctx, outp, n, "f32", it % size, "sum", input=inp,
                                max_segment_bytes=256 << 10)
    hip_rt.synchronize()
    res.append(hip_rt.d2h(outp, like))
    modes.append(ctx.last_mode()["interp_slices"])
ctx.close()
np.save(out, np.array(res))
np.save(out + ".slices.npy", np.array(modes))
'''


@pytest.mark.parametrize("kind,P,env", [
    ("bcube", 4, {}),                                   # 2 x 2: recursive halving shape (mesh: tree fold)
    ("bcube", 6, {}),                                   # 2 x 3 (mesh: pairwise folds)
    ("bcube", 4, {"GLOO_AMD_MESH": "0"}),               # the reference's exchange route
    ("bcube", 3, {"GLOO_AMD_MESH": "0", "GLOO_AMD_INTERP": "0"}),
    ("reduce", 4, {}),
    ("reduce", 5, {"GLOO_AMD_MESH": "0"}),
    ("reduce", 3, {"GLOO_AMD_MESH": "0", "GLOO_AMD_GRAPH": "0"}),
    ("ring", 4, {}),                                    # new-style RING, mesh route
    ("ring", 3, {"GLOO_AMD_MESH": "0"}),
    # the sliced interpreter (executor.h), ragged slices, local steps split
    ("ring", 4, {"GLOO_AMD_TEST_N": "1001", "GLOO_AMD_INTERP_SLICE_BYTES": "128"}),
    ("bcube", 6, {"GLOO_AMD_TEST_N": "999", "GLOO_AMD_INTERP_SLICE_BYTES": "64"}),
    ("reduce", 4, {"GLOO_AMD_TEST_N": "4097", "GLOO_AMD_INTERP_SLICE_BYTES": "256"}),
    ("ring", 4, {"GLOO_AMD_INTERP": "0"}),              # graph replay / eager route at the default size
    # many segments: more interpreter steps than the device list holds, so no
    # rank may propose the sliced form (it has no fallback route)
    ("reduce", 4, {"GLOO_AMD_MESH": "0", "GLOO_AMD_TEST_N": "8000000"}),
    ("ring", 4, {"GLOO_AMD_MESH": "0", "GLOO_AMD_TEST_N": "8000000"}),
])
def test_processes(torch, kind, P, env):
    """Ranks as processes (device signalling unless overridden; inboxes over
    HIP IPC), alternating buffer sets so the cached schedule is rebound and
    re-captured; the root rotates for reduce.  Inputs (rank+1)*(it+1): exact
    sums (it+1)*P(P+1)/2."""
    with tempfile.TemporaryDirectory() as d:
        w = os.path.join(d, "w.py")
        open(w, "w").write(WORKER)
        e = dict(os.environ, GLOO_AMD_ROOT=ROOT, **env)
        procs = [subprocess.Popen([sys.executable, w, str(r), str(P), "file:" + os.path.join(d, "s"), kind,
                                   os.path.join(d, f"o{r}.npy")], env=e) for r in range(P)]
        assert [p.wait(timeout=300) for p in procs] == [0] * P
        ys = [np.load(os.path.join(d, f"o{r}.npy")) for r in range(P)]
        slices = [np.load(os.path.join(d, f"o{r}.npy.slices.npy")) for r in range(P)]
    if env.get("GLOO_AMD_TEST_N") == "8000000":
        # the step list would overflow the device list: slicing refused
        assert all((s == 0).all() for s in slices), slices
    elif "GLOO_AMD_INTERP_SLICE_BYTES" in env:
        # the interpreter runs (sliced where the plan allows: the 2 x 3 BCUBE
        # mesh's pairwise folds through arena temporaries keep one workgroup)
        assert all((s >= 1).all() for s in slices), slices
        if kind != "bcube":
            assert all((s > 1).all() for s in slices), slices
    for it in range(ys[0].shape[0]):
        want = (it + 1) * P * (P + 1) / 2
        if kind in ("bcube", "ring"):
            for r in range(P):
                assert (ys[r][it] == want).all(), (r, it)
        else:
            assert (ys[it % P][it] == want).all(), it


STAGING_WORKER = r'''
import os, sys, json, numpy as np
sys.path.insert(0, os.environ["GLOO_AMD_ROOT"])
import torch, gloo_amd
rank, size, store = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
torch.cuda.set_device(0)
n = 50_000
ctx = gloo_amd.Context(rank, size, store, device=0, timeout_ms=60000)
res = []
for it, staged in enumerate([False, True, True, False]):
    # a second output "on another GPU" (GLOO_AMD_FORCE_STAGING marks it so)
    # from the second call on: the cached sliced schedule is rebound to it
    if staged:
        os.environ["GLOO_AMD_FORCE_STAGING"] = "1"
    else:
        os.environ.pop("GLOO_AMD_FORCE_STAGING", None)
    outs = [torch.full((n,), float((rank + 1) * (j + 1) * (it + 1)), device="cuda:0") for j in range(2)]
    torch.cuda.synchronize()
    gloo_amd.allreduce(ctx, [o.data_ptr() for o in outs], n, "f32", "sum")
    m = ctx.last_mode()
    res.append({"vals": [float(o[0]) for o in outs] + [float(o[-1]) for o in outs],
                "ok": all(bool((o == o[0]).all()) for o in outs), "slices": m["interp_slices"]})
ctx.close()
print("RESULT" + json.dumps(res), flush=True)
'''


def test_processes_sliced_rebind_to_staged_output(torch):
    """a cached sliced schedule rebound to an output on another GPU
    of the process used to throw on that rank only (its peers then waited
    out the timeout).  Now the step list runs over a local staging copy of
    that output and keeps the sliced form; a later local rebinding runs
    without staging again."""
    P = 2
    with tempfile.TemporaryDirectory() as d:
        w = os.path.join(d, "w.py")
        open(w, "w").write(STAGING_WORKER)
        e = dict(os.environ, GLOO_AMD_ROOT=ROOT)
        e.pop("GLOO_AMD_FORCE_STAGING", None)
        procs = [subprocess.Popen([sys.executable, w, str(r), str(P), "file:" + os.path.join(d, "s")], env=e,
                                  stdout=subprocess.PIPE, text=True) for r in range(P)]
        outs = [p.communicate(timeout=240)[0] for p in procs]
        assert [p.returncode for p in procs] == [0] * P
    for r in range(P):
        res = json.loads(outs[r].split("RESULT", 1)[1])
        for it, x in enumerate(res):
            want = (it + 1) * 3 * P * (P + 1) / 2
            assert x["ok"] and x["vals"] == [want] * 4, (r, it, x)
            assert x["slices"] > 1, (r, it, x)
