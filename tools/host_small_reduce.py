"""MEASUREMENT: small host-resident chunks, GPU zero-copy kernel against a CPU
reduce.

The reference reduces host-resident chunks below 256 KiB on the CPU
(gloo/algorithm.cc:16 kOnDeviceThreshold, used at
gloo/cuda_allreduce_halving_doubling.cc:480).  In this library's HOST
workspace the accumulator is the caller's DEVICE buffer and the peer's chunk
lands in pinned host memory; the REDUCE step is one kernel that reads the
host chunk in place (zero-copy).  The CPU alternative for the same step must
bring the accumulator to the host and back:

  zero_copy  gloo_hip_reduce(dev_acc, mapped host chunk), stream synchronise
  cpu        D2H of the accumulator range, dst += src on the host (numpy,
             one thread, as Gloo's sum<float>), H2D back, synchronise
  cpu_host_only  dst += src with both operands already on the host (what the
             reference's CPU path costs when nothing has to move; a lower bound)

One JSON line per size: p50 microseconds of each over `iters` repetitions.
Usage: python tools/host_small_reduce.py [iters]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import gloo_amd as hip
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = torch.cuda.current_stream(dev)
    hiprt = ctypes.CDLL("libamdhip64.so")
    for kib in (1, 4, 16, 64, 256, 1024):
        n = kib * 1024 // 4
        h_src = torch.empty(n, dtype=torch.float32, pin_memory=True).uniform_(-1, 1)
        h_acc = torch.empty(n, dtype=torch.float32, pin_memory=True)
        d_acc = torch.empty(n, dtype=torch.float32, device=dev).uniform_(-1, 1)
        ref = (d_acc.cpu() + h_src).numpy()
        p = ctypes.c_void_p()
        assert hiprt.hipHostGetDevicePointer(ctypes.byref(p), ctypes.c_void_p(h_src.data_ptr()), 0) == 0
        hs = p.value
        a_np, s_np = h_acc.numpy(), h_src.numpy()

        def zero_copy():
            hip.reduce_ptr("sum", "f32", d_acc.data_ptr(), hs, n, s.cuda_stream)
            s.synchronize()

        def cpu():
            h_acc.copy_(d_acc)  # D2H, synchronous
            np.add(a_np, s_np, out=a_np)
            d_acc.copy_(h_acc)  # H2D
            s.synchronize()

        def cpu_host_only():
            np.add(a_np, s_np, out=a_np)

        out = {"bytes": n * 4}
        for name, fn in (("zero_copy", zero_copy), ("cpu", cpu), ("cpu_host_only", cpu_host_only)):
            base = d_acc.clone()
            for _ in range(5):
                fn()
            ts = []
            for _ in range(iters):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            ts.sort()
            out[name + "_us_p50"] = round(ts[len(ts) // 2] * 1e6, 2)
            d_acc.copy_(base)
        # both GPU-side variants give the IEEE sum (one reduction from a known state)
        base = d_acc.clone()
        zero_copy()
        out["zero_copy_exact"] = bool(np.array_equal(d_acc.cpu().numpy(), ref))
        d_acc.copy_(base)
        cpu()
        out["cpu_exact"] = bool(np.array_equal(d_acc.cpu().numpy(), ref))
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
