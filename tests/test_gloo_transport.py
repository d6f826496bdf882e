"""The xGMI transport as a gloo::transport::Device
(gloo_amd/include/gloo_amd/gloo_transport.h).

CPU: gloo_hip_context_create_kv bootstraps the library's context over a
caller's key/value store (the gloo::IStore that
transport::Context::createAndConnectAllPairs receives,
gloo/transport/context.cc:26-89) — Python threads as ranks, a dict as the
store; a store that times out surfaces as IoException (GLOO_HIP_EIO).

GPU: oracle/_ref/transport_test, a Gloo program built against the reference's
headers and objects: connectFullMesh over the hip device, a device
ring-chunked allreduce on its bound buffers (threads, and processes sharing
receive buffers over HIP IPC), gloo::HipAllreduce* on that context, the
reference's own AllreduceRingChunked / AllreduceHalvingDoubling templates and
rendezvous::ContextFactory over it, IoException, four ring-chunked instances
live at once (12 slots per pair), and the unbound buffers: the reference's own
gloo::allreduce (RING, BCUBE), gloo::allgather and gloo::reduce on host
buffers over this transport, recv-from-any, per-slot ordering with device
buffers, abort.  Processes: the device ring-chunked with the reference's
host-word notification buffers (&dummy_) and gloo::allreduce on host
buffers between processes.  Closed form of gloo/test/base_test.h:184-236.
"""
import ctypes
import os
import subprocess
import tempfile
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRANSPORT_TEST = os.path.join(ROOT, "oracle", "_ref", "transport_test")

KV_SET = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t)
KV_GET = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p,
                          ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t))


class DictStore:
    """set / wait+get over a dict shared by Python threads (a HashStore)."""

    def __init__(self):
        self.d = {}
        self.cv = threading.Condition()
        self.sets = 0

        def set_(user, key, data, n):
            with self.cv:
                self.d[key] = ctypes.string_at(data, n)
                self.sets += 1
                self.cv.notify_all()
            return 0

        def get(user, key, timeout_ms, out, cap, length):
            deadline = time.monotonic() + timeout_ms / 1e3
            with self.cv:
                while key not in self.d:
                    left = deadline - time.monotonic()
                    if left <= 0:
                        return -5
                    self.cv.wait(left)
                v = self.d[key]
            length[0] = len(v)
            if len(v) <= cap:
                ctypes.memmove(out, v, len(v))
            return 0

        self.set_cb, self.get_cb = KV_SET(set_), KV_GET(get)


def _bind(lib):
    lib.gloo_hip_context_create_kv.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, KV_SET,
                                               KV_GET, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]
    lib.gloo_hip_context_destroy.argtypes = [ctypes.c_void_p]


def test_context_bootstrap_over_caller_store():
    import gloo_amd
    lib = gloo_amd.lib
    _bind(lib)
    P = 3
    store = DictStore()
    rcs, handles = [None] * P, [None] * P

    def body(r):
        h = ctypes.c_void_p()
        rcs[r] = lib.gloo_hip_context_create_kv(r, P, 0, 10000, store.set_cb, store.get_cb, None, ctypes.byref(h))
        handles[r] = h

    ts = [threading.Thread(target=body, args=(r,)) for r in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert rcs == [0] * P, lib.gloo_hip_last_error()
    assert store.sets >= P
    for h in handles:
        assert lib.gloo_hip_context_destroy(h) == 0


def test_store_timeout_is_io_exception():
    import gloo_amd
    lib = gloo_amd.lib
    _bind(lib)
    store = DictStore()  # the peer never shows up
    h = ctypes.c_void_p()
    rc = lib.gloo_hip_context_create_kv(0, 2, 0, 300, store.set_cb, store.get_cb, None, ctypes.byref(h))
    assert rc == -5, rc
    assert b"IoException" in lib.gloo_hip_last_error()


def test_transport_header_is_gloo_side_only():
    """gloo_transport.h is compiled by the Gloo program; the product sources
    never include it (nor any gloo/ header)."""
    src = os.path.join(ROOT, "gloo_amd", "csrc")
    for f in os.listdir(src):
        text = open(os.path.join(src, f)).read()
        assert "gloo_transport.h" not in text, f


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_transport_program_on_gpu():
    pytest.importorskip("torch")
    if not os.path.exists(TRANSPORT_TEST):
        pytest.skip("oracle/_ref/transport_test not built (needs /root/reference at build time)")
    r = subprocess.run([TRANSPORT_TEST], capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith(("ok", "FAIL"))]
    assert lines and all(l.startswith("ok") for l in lines), r.stdout
    assert len(lines) >= 45
    names = " ".join(lines)
    for case in ("many_live/", "ref_allreduce_ring_host/", "ref_allreduce_bcube_host/", "ref_allgather_host/",
                 "ref_reduce_host/", "unbound_recv_from_any/", "unbound_order_device/", "unbound_abort/"):
        assert case in names, case


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_transport_processes_on_gpu():
    """Ranks as processes: receive buffers cross over HIP IPC; the store is
    the reference's FileStore."""
    pytest.importorskip("torch")
    if not os.path.exists(TRANSPORT_TEST):
        pytest.skip("oracle/_ref/transport_test not built (needs /root/reference at build time)")
    P, n = 3, 100003
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([TRANSPORT_TEST, "proc", str(r), str(P), d, str(n)], stdout=subprocess.PIPE,
                                  stderr=subprocess.STDOUT, text=True) for r in range(P)]
        outs = []
        for p in procs:
            try:
                out, _ = p.communicate(timeout=240)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            outs.append((p.returncode, out))
    for r, (rc, out) in enumerate(outs):
        assert rc == 0 and f"ok   proc rank {r}" in out, out[-3000:]
