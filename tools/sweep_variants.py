#!/usr/bin/env python3
"""Tuning sweep (GPU): fp32 SUM kernel variants at 64 MiB, and the chunk-size
regime 1 KiB .. 1 GiB for the default kernel (latency vs bandwidth, the sizes
halving-doubling steps produce, BASELINE config 4).  Prints one JSON line per
measurement.  Not part of the graded bench; its outputs go to profiles/."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import gloo_amd as hip  # noqa: E402

VARIANTS = {0: "default: unroll2 block512 nt-load nt-store", 1: "unroll2 block256", 2: "unroll4 block256",
            3: "unroll1 block512", 4: "unroll2 block512 nt-load plain-store", 5: "unroll2 block1024",
            6: "unroll1 block1024", 7: "unroll2 block512 store nt|sc1", 8: "unroll3 block512"}


def bench(n, steps, pairs, variant=0):
    dev = torch.device("cuda:0")
    hip.set_variant(variant)
    bufs = [(torch.rand(n, device=dev), torch.rand(n, device=dev)) for _ in range(pairs)]
    s = torch.cuda.current_stream().cuda_stream
    for i in range(10):
        d, x = bufs[i % pairs]
        hip.reduce_ptr("sum", "f32", d.data_ptr(), x.data_ptr(), n, s)
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for i in range(steps):
        d, x = bufs[i % pairs]
        evs[i][0].record()
        hip.reduce_ptr("sum", "f32", d.data_ptr(), x.data_ptr(), n, s)
        evs[i][1].record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in evs)
    mean = sum(ts) / len(ts)
    med = ts[len(ts) // 2]
    hip.set_variant(0)
    del bufs
    torch.cuda.empty_cache()
    return mean, med


def bench_misaligned(n, steps, pairs, src_off_elems, dtype_bytes=4):
    """dst 16-B aligned, src shifted by src_off_elems elements: the
    relatively-misaligned case an arbitrary Gloo chunk offset produces."""
    dev = torch.device("cuda:0")
    bufs = [(torch.rand(n + 8, device=dev), torch.rand(n + 8, device=dev)) for _ in range(pairs)]
    s = torch.cuda.current_stream().cuda_stream
    es = dtype_bytes
    for i in range(5):
        d, x = bufs[i % pairs]
        hip.reduce_ptr("sum", "f32", d.data_ptr(), x.data_ptr() + src_off_elems * es, n, s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(steps):
        d, x = bufs[i % pairs]
        hip.reduce_ptr("sum", "f32", d.data_ptr(), x.data_ptr() + src_off_elems * es, n, s)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / steps
    del bufs
    torch.cuda.empty_cache()
    return us


def bench_finegrained_src(n, steps, pairs):
    """dst coarse-grained (hipMalloc), src in fine-grained device memory
    (hipExtMallocWithFlags(hipDeviceMallocFinegrained)) — the inbox arenas a
    peer GPU writes over xGMI."""
    import ctypes
    hiprt = ctypes.CDLL("libamdhip64.so")
    hiprt.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hiprt.hipFree.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    dsts = [torch.rand(n, device=dev) for _ in range(pairs)]
    srcs = []
    for _ in range(pairs):
        p = ctypes.c_void_p()
        assert hiprt.hipExtMallocWithFlags(ctypes.byref(p), n * 4, 0x1) == 0  # hipDeviceMallocFinegrained
        srcs.append(p.value)
    s = torch.cuda.current_stream().cuda_stream
    for i in range(5):
        hip.reduce_ptr("sum", "f32", dsts[i % pairs].data_ptr(), srcs[i % pairs], n, s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(steps):
        hip.reduce_ptr("sum", "f32", dsts[i % pairs].data_ptr(), srcs[i % pairs], n, s)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / steps
    for p in srcs:
        hiprt.hipFree(p)
    del dsts
    torch.cuda.empty_cache()
    return us


def main():
    n = 16 << 20
    us = bench_finegrained_src(n, 300, 6)
    print(json.dumps({"sweep": "finegrained_src", "us_mean": round(us, 2),
                      "GBs": round(3 * n * 4 / (us / 1e3) / 1e9, 1)}), flush=True)
    for off in (0, 1, 2, 3):
        us = bench_misaligned(n, 300, 6, off)
        print(json.dumps({"sweep": "relative_misalignment", "src_offset_elems": off, "us_mean": round(us, 2),
                          "GBs": round(3 * n * 4 / (us / 1e3) / 1e9, 1)}), flush=True)
    for v in VARIANTS:
        mean, med = bench(n, 300, 6, v)
        print(json.dumps({"sweep": "variant", "variant": v, "name": VARIANTS[v],
                          "us_mean": round(mean * 1e3, 2), "us_median": round(med * 1e3, 2),
                          "GBs_mean": round(3 * n * 4 / (mean / 1e3) / 1e9, 1)}), flush=True)
    for lg in range(8, 29, 2):  # 1 KiB .. 1 GiB of fp32 per operand
        n = 1 << lg
        pairs = max(2, min(64, (768 << 20) // (8 * n)))
        steps = 200 if n < (1 << 26) else 30
        mean, med = bench(n, steps, pairs)
        print(json.dumps({"sweep": "size", "bytes": 4 * n, "us_mean": round(mean * 1e3, 2),
                          "us_median": round(med * 1e3, 2),
                          "GBs_median": round(3 * n * 4 / (med / 1e3) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
