#!/usr/bin/env python3
"""Probe (measurement tool, not product): what the HIP runtime does when an
IPC-exported block is freed while a peer process still maps it.

  exporter: A = hipMalloc 1 GiB, export, wait for the importer's mapping;
            hipFree(A) (timed); B = hipMalloc 512 MiB, export (rc?), report
            addresses; tell the importer; wait for its close;
            C = hipMalloc 512 MiB, export (rc?).
  importer: map A, signal; wait for "freed"; read A's first word through the
            old mapping; close (timed); signal.
usage: ipc_free_probe.py  (spawns both; JSON lines on stdout)"""
import ctypes
import json
import os
import subprocess
import sys
import tempfile
import time

HIP = "libamdhip64.so.7"


class Handle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * 64)]


def rt():
    L = ctypes.CDLL(HIP)
    L.hipIpcGetMemHandle.argtypes = [ctypes.POINTER(Handle), ctypes.c_void_p]
    L.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), Handle, ctypes.c_uint]
    L.hipIpcCloseMemHandle.argtypes = [ctypes.c_void_p]
    L.hipFree.argtypes = [ctypes.c_void_p]
    L.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    L.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    L.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return L


def put(d, name, data=b"1"):
    with open(os.path.join(d, name + ".tmp"), "wb") as f:
        f.write(data)
    os.rename(os.path.join(d, name + ".tmp"), os.path.join(d, name))


def wait_file(d, name, limit):
    t0 = time.time()
    path = os.path.join(d, name)
    while not os.path.exists(path):
        if time.time() - t0 > limit:
            return False
        time.sleep(0.01)
    return True


def alloc_export(L, nbytes, fill):
    p = ctypes.c_void_p()
    rc = L.hipMalloc(ctypes.byref(p), nbytes)
    if rc:
        return None, None, rc
    L.hipMemset(p, fill, nbytes)
    L.hipDeviceSynchronize()
    h = Handle()
    return p, h, L.hipIpcGetMemHandle(ctypes.byref(h), p)


def exporter(d):
    L = rt()
    L.hipSetDevice(0)
    a, ha, rc = alloc_export(L, 1 << 30, 0xAA)
    assert rc == 0, rc
    put(d, "handle", ctypes.string_at(ctypes.byref(ha), 64))
    assert wait_file(d, "imported", 60)
    t0 = time.time()
    rc_free = L.hipFree(a)
    t_free = time.time() - t0
    b, hb, rc_b = alloc_export(L, 512 << 20, 0x55)
    print(json.dumps({"exporter": "freed A while mapped, exported B", "hipFree_rc": rc_free,
                      "hipFree_s": round(t_free, 4), "A": hex(a.value), "B": hex(b.value) if b else None,
                      "B_inside_A": bool(b and a.value <= b.value < a.value + (1 << 30)),
                      "export_B_rc": rc_b}), flush=True)
    put(d, "freed")
    assert wait_file(d, "closed", 60)
    c, hc, rc_c = alloc_export(L, 512 << 20, 0x33)
    print(json.dumps({"exporter": "after the importer closed A, exported C", "C": hex(c.value) if c else None,
                      "C_inside_A": bool(c and a.value <= c.value < a.value + (1 << 30)),
                      "export_C_rc": rc_c}), flush=True)
    for x in (b, c):
        if x:
            L.hipFree(x)


def importer(d):
    L = rt()
    L.hipSetDevice(0)
    assert wait_file(d, "handle", 60)
    h = Handle.from_buffer_copy(open(os.path.join(d, "handle"), "rb").read())
    m = ctypes.c_void_p()
    rc = L.hipIpcOpenMemHandle(ctypes.byref(m), h, 1)
    put(d, "imported")
    ok = wait_file(d, "freed", 30)
    seen = ctypes.c_uint64(0)
    rc_read = L.hipMemcpy(ctypes.byref(seen), m, 8, 2) if rc == 0 else None
    t0 = time.time()
    rc2 = L.hipIpcCloseMemHandle(m) if rc == 0 else None
    print(json.dumps({"importer": "read A after its free, closed", "open_rc": rc, "read_rc": rc_read,
                      "first_word": hex(seen.value), "close_rc": rc2, "close_s": round(time.time() - t0, 4),
                      "saw_freed": ok}), flush=True)
    put(d, "closed")


if __name__ == "__main__":
    if len(sys.argv) > 2:
        (exporter if sys.argv[1] == "e" else importer)(sys.argv[2])
        sys.exit(0)
    with tempfile.TemporaryDirectory() as d:
        ps = [subprocess.Popen([sys.executable, __file__, w, d]) for w in ("e", "i")]
        rcs = [p.wait(timeout=120) for p in ps]
        print(json.dumps({"rcs": rcs}), flush=True)
