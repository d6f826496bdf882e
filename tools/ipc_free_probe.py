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


def rt():
    L = ctypes.CDLL(HIP)
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
    h = (ctypes.c_char * 64)()
    assert L.hipIpcGetMemHandle(h, p) == 0
    open(os.path.join(d, "handle.tmp"), "wb").write(bytes(h))
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
    h2 = (ctypes.c_char * 64)()
    L.hipIpcGetMemHandle(h2, q)
    print(json.dumps({"exporter": "freed", "hipFree_rc": rc, "hipFree_s": round(t_free, 4),
                      "old": hex(p.value), "new": hex(q.value), "same_address": p.value == q.value,
                      "same_handle": bytes(h) == bytes(h2)}), flush=True)
    open(os.path.join(d, "freed"), "w").write("1")
    wait_file(os.path.join(d, "closed"), 60)
    L.hipFree(q)


def importer(d):
    L = rt()
    L.hipSetDevice(0)
    assert wait_file(os.path.join(d, "handle"), 60)
    h = (ctypes.c_char * 64).from_buffer_copy(open(os.path.join(d, "handle"), "rb").read())
    m = ctypes.c_void_p()
    rc = L.hipIpcOpenMemHandle(ctypes.byref(m), h, ctypes.c_uint(1))
    open(os.path.join(d, "imported"), "w").write("1")
    ok = wait_file(os.path.join(d, "freed"), 30)
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
