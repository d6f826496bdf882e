#!/usr/bin/env python3
"""Probe (measurement tool, not product): does hipFree of an IPC-exported
block block while a peer process still has it mapped?  And may the exporter
free a block, allocate again, and hand out a NEW handle at that address?

  exporter: hipMalloc 64 MiB, export, wait for the importer's mapping,
            hipFree (timed, watchdog prints every 2 s), allocate again and
            report the new address, then tell the importer.
  importer: map, signal, wait for "freed" (at most 30 s), close, report.
usage: ipc_free_probe.py  (spawns both; JSON lines on stdout)"""
import ctypes
import json
import os
import subprocess
import sys
import tempfile
import threading
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
    return L


def wait_file(path, limit):
    t0 = time.time()
    while not os.path.exists(path):
        if time.time() - t0 > limit:
            return False
        time.sleep(0.01)
    return True


def exporter(d):
    L = rt()
    L.hipSetDevice(0)
    p = ctypes.c_void_p()
    assert L.hipMalloc(ctypes.byref(p), ctypes.c_size_t(64 << 20)) == 0
    L.hipMemset(p, 0xAA, ctypes.c_size_t(64 << 20))
    L.hipDeviceSynchronize()
    h = Handle()
    assert L.hipIpcGetMemHandle(ctypes.byref(h), p) == 0
    open(os.path.join(d, "handle.tmp"), "wb").write(bytes(h.reserved))
    os.rename(os.path.join(d, "handle.tmp"), os.path.join(d, "handle"))
    assert wait_file(os.path.join(d, "imported"), 60)
    stop = [False]

    def dog():
        t0 = time.time()
        while not stop[0]:
            time.sleep(2)
            if not stop[0]:
                print(json.dumps({"exporter": "hipFree still blocked", "s": round(time.time() - t0, 1)}), flush=True)
    threading.Thread(target=dog, daemon=True).start()
    t0 = time.time()
    rc = L.hipFree(p)
    stop[0] = True
    t_free = time.time() - t0
    q = ctypes.c_void_p()
    assert L.hipMalloc(ctypes.byref(q), ctypes.c_size_t(64 << 20)) == 0
    L.hipMemset(q, 0x55, ctypes.c_size_t(64 << 20))
    L.hipDeviceSynchronize()
    h2 = Handle()
    L.hipIpcGetMemHandle(ctypes.byref(h2), q)
    open(os.path.join(d, "handle2.tmp"), "wb").write(bytes(h2.reserved))
    os.rename(os.path.join(d, "handle2.tmp"), os.path.join(d, "handle2"))
    print(json.dumps({"exporter": "freed", "hipFree_rc": rc, "hipFree_s": round(t_free, 4),
                      "old": hex(p.value), "new": hex(q.value), "same_address": p.value == q.value,
                      "same_handle": bytes(h.reserved) == bytes(h2.reserved)}), flush=True)
    open(os.path.join(d, "freed"), "w").write("1")
    wait_file(os.path.join(d, "closed"), 60)
    L.hipFree(q)


def importer(d):
    L = rt()
    L.hipSetDevice(0)
    assert wait_file(os.path.join(d, "handle"), 60)
    h = Handle.from_buffer_copy(open(os.path.join(d, "handle"), "rb").read())
    m = ctypes.c_void_p()
    rc = L.hipIpcOpenMemHandle(ctypes.byref(m), h, 1)
    open(os.path.join(d, "imported"), "w").write("1")
    ok = wait_file(os.path.join(d, "freed"), 12)
    # while the first mapping is still open: the exporter's new block at the
    # same address, through its own (different?) handle
    seen = ctypes.c_uint64(0)
    rc3 = rc4 = None
    if ok and wait_file(os.path.join(d, "handle2"), 5):
        h2 = Handle.from_buffer_copy(open(os.path.join(d, "handle2"), "rb").read())
        m2 = ctypes.c_void_p()
        rc3 = L.hipIpcOpenMemHandle(ctypes.byref(m2), h2, 1)
        if rc3 == 0:
            L.hipMemcpy(ctypes.byref(seen), m2, ctypes.c_size_t(8), 2)
            rc4 = L.hipIpcCloseMemHandle(m2)
        print(json.dumps({"importer": "second import", "open_rc": rc3, "first_word": hex(seen.value),
                          "same_mapping_as_first": m2.value == m.value if rc3 == 0 else None,
                          "close_rc": rc4}), flush=True)
    t0 = time.time()
    rc2 = L.hipIpcCloseMemHandle(m)
    print(json.dumps({"importer": "closed", "open_rc": rc, "close_rc": rc2, "close_s": round(time.time() - t0, 4),
                      "saw_freed_before_close": ok}), flush=True)
    open(os.path.join(d, "closed"), "w").write("1")


if __name__ == "__main__":
    if len(sys.argv) > 2:
        (exporter if sys.argv[1] == "e" else importer)(sys.argv[2])
        sys.exit(0)
    with tempfile.TemporaryDirectory() as d:
        ps = [subprocess.Popen([sys.executable, __file__, w, d]) for w in ("e", "i")]
        rcs = [p.wait(timeout=120) for p in ps]
        print(json.dumps({"rcs": rcs}), flush=True)
