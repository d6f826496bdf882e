"""The Gloo-surface bridge (gloo_amd/include/gloo_amd/gloo_bridge.h).

CPU: gloo_hip_context_create_ex bootstraps the library's context with a
caller-supplied all-gather and nothing else (no store, no second
rendezvous) — exercised here with Python threads as ranks and a Python
all-gather; a failing all-gather surfaces as IoException (GLOO_HIP_EIO).

GPU: oracle/_ref/bridge_test, a Gloo program built against the reference's
own headers and objects (oracle/Makefile), constructs gloo::HipAllreduce*<T>
from its gloo::Context (threads over the reference's TCP transport) and
checks the closed form of gloo/test/base_test.h:184-236 — ring, ring-chunked,
halving-doubling (+ pipelined), multi-pointer, user streams, fp16, the host
workspace, reduce-scatter and the IoException of a silent peer.
"""
import ctypes
import os
import subprocess
import threading

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BRIDGE_TEST = os.path.join(ROOT, "oracle", "_ref", "bridge_test")

ALLGATHER = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)


class ThreadAllgather:
    """An all-gather among P Python threads (the role gloo::allgather plays
    over a gloo::Context's pairs)."""

    def __init__(self, P):
        self.P = P
        self.barrier = threading.Barrier(P)
        self.blocks = [None] * P
        self.calls = [0] * P

    def fn(self, rank, fail=False):
        def cb(user, inp, out, block):
            if fail:
                return 1
            self.calls[rank] += 1
            self.blocks[rank] = ctypes.string_at(inp, block)
            self.barrier.wait()
            ctypes.memmove(out, b"".join(self.blocks), block * self.P)
            self.barrier.wait()
            return 0
        return ALLGATHER(cb)


def _bind(lib):
    lib.gloo_hip_context_create_ex.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ALLGATHER,
                                               ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]
    lib.gloo_hip_context_destroy.argtypes = [ctypes.c_void_p]


def test_context_bootstrap_over_caller_allgather():
    import gloo_amd
    lib = gloo_amd.lib
    _bind(lib)
    P = 3
    ag = ThreadAllgather(P)
    cbs = [ag.fn(r) for r in range(P)]
    rcs, handles = [None] * P, [None] * P

    def body(r):
        h = ctypes.c_void_p()
        rcs[r] = lib.gloo_hip_context_create_ex(r, P, 0, 10000, cbs[r], None, ctypes.byref(h))
        handles[r] = h

    ts = [threading.Thread(target=body, args=(r,)) for r in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert rcs == [0] * P
    # connect = one all-gather for the control block's name + one barrier
    assert ag.calls == [2] * P
    for h in handles:
        assert lib.gloo_hip_context_destroy(h) == 0


def test_failed_allgather_is_io_exception():
    import gloo_amd
    lib = gloo_amd.lib
    _bind(lib)
    cb = ThreadAllgather(1).fn(0, fail=True)
    h = ctypes.c_void_p()
    rc = lib.gloo_hip_context_create_ex(0, 2, 0, 1000, cb, None, ctypes.byref(h))
    assert rc == -5, rc
    assert b"IoException" in lib.gloo_hip_last_error()


def test_bridge_header_is_gloo_side_only():
    """libgloo_amd.so must not link the reference: the bridge is a header the
    Gloo side compiles, and the product sources never include gloo/ headers."""
    src = os.path.join(ROOT, "gloo_amd", "csrc")
    for f in os.listdir(src):
        text = open(os.path.join(src, f)).read()
        assert '#include "gloo/' not in text, f
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(ROOT, "gloo_amd", "libgloo_amd.so")],
                         capture_output=True, text=True).stdout
    assert "_ZN4gloo" not in out  # no symbol of namespace gloo (the reference's)


def test_bridge_bootstrap_cpu():
    """The bridge's BootstrapContext (gloo::allgather over the reference's
    own TCP pairs) creates and destroys the library context — no GPU call."""
    if not os.path.exists(BRIDGE_TEST):
        pytest.skip("oracle/_ref/bridge_test not built (needs /root/reference at build time)")
    r = subprocess.run([BRIDGE_TEST, "bootstrap_cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("ok   bootstrap_cpu") == 4, r.stdout


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bridge_program_on_gpu():
    pytest.importorskip("torch")
    if not os.path.exists(BRIDGE_TEST):
        pytest.skip("oracle/_ref/bridge_test not built (needs /root/reference at build time)")
    r = subprocess.run([BRIDGE_TEST, "/"], capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith(("ok", "FAIL"))]
    assert lines and all(l.startswith("ok") for l in lines), r.stdout
    assert len(lines) >= 30
