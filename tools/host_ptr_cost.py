"""MEASUREMENT ONLY: host-side cost of the calls gloo_hip_reduce_staged can use
to tell whether a host buffer is pinned and mapped (hipHostGetDevicePointer,
hipPointerGetAttributes), on torch pin_memory() tensors."""
import ctypes
import json
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
t = torch.empty(1 << 24, dtype=torch.float32, pin_memory=True)
p = ctypes.c_void_p()
attr = (ctypes.c_char * 256)()
torch.cuda.synchronize()
for name, fn in (("hipHostGetDevicePointer",
                  lambda: hip.hipHostGetDevicePointer(ctypes.byref(p), ctypes.c_void_p(t.data_ptr()), 0)),
                 ("hipPointerGetAttributes",
                  lambda: hip.hipPointerGetAttributes(ctypes.byref(attr), ctypes.c_void_p(t.data_ptr())))):
    for _ in range(10):
        fn()
    t0 = time.perf_counter()
    for _ in range(1000):
        rc = fn()
    us = (time.perf_counter() - t0) * 1e6 / 1000
    print(json.dumps({"call": name, "us": round(us, 2), "rc": rc, "same_address": p.value == t.data_ptr()}))
