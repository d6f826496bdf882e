"""GPU: caller-supplied device reductions (gloo_hip_register_op) — the
reference's ReductionType::CUSTOM with a user function
(gloo/algorithm.h:49-95) and the new-style `Func` (gloo/allreduce.h:36) on
device memory.  The op here is bytewise XOR (tests/custom_op/xor_op.hip): not
a built-in, exact and order-independent, so every schedule must return the
XOR of all ranks' inputs; the function is called for every REDUCE / FOLD
step, the fused and interpreted kernels are never used."""
import ctypes
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import uuid

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
XOR_LIB = os.path.join(ROOT, "tests", "custom_op", "libxor_op.so")


@pytest.fixture(scope="module")
def torch():
    t = pytest.importorskip("torch")
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.fixture(scope="module")
def xor_op(torch):
    import gloo_amd
    lib = ctypes.CDLL(XOR_LIB)
    lib.xor_op_calls.restype = ctypes.c_ulonglong
    fn = ctypes.cast(lib.xor_op_fn, ctypes.c_void_p).value
    user = ctypes.addressof(ctypes.c_int.in_dll(lib, "xor_elem_size_4"))
    op = gloo_amd.register_op(fn, user)
    assert op >= 1000
    return op, lib


def test_reduce3_and_multi(torch, xor_op):
    import gloo_amd
    op, lib = xor_op
    rng = np.random.default_rng(1)
    a, b, c = (rng.integers(-2**31, 2**31, 100_003, dtype=np.int64).astype(np.int32) for _ in range(3))
    ta, tb, tc = (torch.from_numpy(x).cuda() for x in (a, b, c))
    out = torch.empty_like(ta)
    before = lib.xor_op_calls()
    gloo_amd.reduce3_ptr(op, "i32", out.data_ptr(), ta.data_ptr(), tb.data_ptr(), a.size)
    torch.cuda.synchronize()
    assert (out.cpu().numpy() == (a ^ b)).all()
    gloo_amd.reduce_multi_ptr(op, "i32", ta.data_ptr(), [ta.data_ptr(), tb.data_ptr(), tc.data_ptr()], a.size)
    torch.cuda.synchronize()
    assert (ta.cpu().numpy() == (a ^ b ^ c)).all()
    assert lib.xor_op_calls() - before == 3


@pytest.mark.parametrize("algo,P", [("ring_chunked", 3), ("ring_chunked", 4), ("halving_doubling", 4),
                                    ("halving_doubling", 5), ("ring", 3), ("local", 1), ("bcube", 4),
                                    ("bcube", 9)])
def test_threads(torch, xor_op, algo, P):
    from test_collectives_gpu import run_threads
    op, _ = xor_op
    k = 3 if algo == "local" else 1
    rng = np.random.default_rng(P)
    x = rng.integers(-2**31, 2**31, (P, k, 10_007), dtype=np.int64).astype(np.int32)
    recv = ([3] if P == 9 else [2]) if algo == "bcube" else None  # AllreduceBcube's base
    y = run_threads(torch, algo, op, "i32", x, recv=recv, runs=1)
    want = np.bitwise_xor.reduce(x.reshape(P * k, -1), axis=0)
    for r in range(P):
        for j in range(k):
            assert (y[r, j] == want).all(), (r, j)


def test_reduce_scatter_threads(torch, xor_op):
    from test_collectives_gpu import run_threads
    op, _ = xor_op
    P, n = 5, 10_007
    recv = [n // P + (1 if r < n % P else 0) for r in range(P)]
    x = np.random.default_rng(9).integers(-2**31, 2**31, (P, 1, n), dtype=np.int64).astype(np.int32)
    y = run_threads(torch, "reduce_scatter", op, "i32", x, recv=recv)
    want = np.bitwise_xor.reduce(x[:, 0], axis=0)
    off = 0
    for r in range(P):
        assert (y[r, 0, :recv[r]] == want[off:off + recv[r]]).all(), r
        off += recv[r]


WORKER = r'''
import ctypes, hashlib, json, os, sys, numpy as np
sys.path.insert(0, os.environ["GLOO_AMD_ROOT"])
import torch, gloo_amd
rank, size, store = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
lib = ctypes.CDLL(os.path.join(os.environ["GLOO_AMD_ROOT"], "tests", "custom_op", "libxor_op.so"))
op = gloo_amd.register_op(ctypes.cast(lib.xor_op_fn, ctypes.c_void_p).value,
                          ctypes.addressof(ctypes.c_int.in_dll(lib, "xor_elem_size_4")))
torch.cuda.set_device(0)
n = 1 << 20
x = np.random.default_rng([5, rank]).integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
src = torch.from_numpy(x).cuda()
buf = torch.empty_like(src)
ctx = gloo_amd.Context(rank, size, store, device=0, timeout_ms=60000)
res = {}
for algo in ("ring_chunked", "halving_doubling"):
    a = gloo_amd.Algorithm(ctx, algo, op, "i32", [buf.data_ptr()], n)
    outs, modes = [], []
    for it in range(3):
        buf.copy_(src); torch.cuda.synchronize()
        a.run()
        outs.append(int(np.bitwise_xor.reduce(buf.cpu().numpy().view(np.uint32)[::97])))
        outs.append(hashlib.sha256(buf.cpu().numpy().tobytes()).hexdigest())
        modes.append(a.mode())
    a.close()
    res[algo] = {"outs": outs, "modes": modes}
# new-style allreduce (RING, BCUBE) and reduce with the custom Func
out = torch.empty_like(src)
for kind in ("ring", "bcube"):
    out.fill_(0)
    gloo_amd.allreduce(ctx, [out.data_ptr()], n, "i32", op, inputs=[src.data_ptr()], algorithm=kind)
    res["new_" + kind] = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()
out.fill_(0)
gloo_amd.reduce_to_root(ctx, out.data_ptr(), n, "i32", 0, op, input=src.data_ptr())
res["reduce"] = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest() if rank == 0 else None
ctx.close()
print("RESULT" + json.dumps(res), flush=True)
'''


@pytest.mark.timeout(300)
def test_processes_graph_replay(torch):
    """Ranks as processes (device signalling, IPC arenas): the custom op runs
    on the reference routes, is captured into the replayed hipGraph, and the
    new-style collectives take it as their Func."""
    P, n = 4, 1 << 20
    with tempfile.TemporaryDirectory() as d:
        w = os.path.join(d, "w.py")
        open(w, "w").write(WORKER)
        e = dict(os.environ, GLOO_AMD_ROOT=ROOT)
        procs = [subprocess.Popen([sys.executable, w, str(r), str(P), "file:" + os.path.join(d, "s")], env=e,
                                  stdout=subprocess.PIPE, text=True) for r in range(P)]
        outs = [p.communicate(timeout=280)[0] for p in procs]
        assert [p.returncode for p in procs] == [0] * P
    res = [json.loads(o.split("RESULT", 1)[1]) for o in outs]
    xs = [np.random.default_rng([5, r]).integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32) for r in range(P)]
    want = np.bitwise_xor.reduce(np.stack(xs), axis=0)
    wh = hashlib.sha256(want.tobytes()).hexdigest()
    wsample = int(np.bitwise_xor.reduce(want.view(np.uint32)[::97]))
    for r in range(P):
        for algo in ("ring_chunked", "halving_doubling"):
            o = res[r][algo]["outs"]
            assert o == [wsample, wh] * 3, (r, algo)
            modes = res[r][algo]["modes"]
            assert not any(m["interp"] for m in modes), modes
            assert modes[-1]["graph"], modes
        assert res[r]["new_ring"] == wh and res[r]["new_bcube"] == wh, r
    assert res[0]["reduce"] == wh
