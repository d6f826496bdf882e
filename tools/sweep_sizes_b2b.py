#!/usr/bin/env python3
"""Chunk-size regime under back-to-back launches (the way device-signalled
plans and graph replay issue them), fp32 in-place sum, 64 KiB .. 256 MiB per
operand.  Buffers rotate over a >= 1 GiB footprint so no size is served from
the 256 MiB Infinity Cache.  HIP events over K launches on the launching
stream; run under rocprofv3 --kernel-trace for the per-launch kernel duration
without dispatch gaps.  Config 3's ring chunk is 16 MiB."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import gloo_amd as hip  # noqa: E402

FOOT = 1 << 30


VARIANTS = {0: "default: unroll2 block512 nt-load nt-store", 1: "unroll2 block256", 2: "unroll4 block256",
            3: "unroll1 block512", 4: "unroll2 block512 nt-load plain-store", 5: "unroll2 block1024",
            6: "unroll1 block1024", 7: "unroll2 block512 store nt|sc1", 8: "unroll3 block512",
            9: "pipelined persistent grid<=256", 10: "pipelined grid<=512", 11: "pipelined grid<=1024",
            12: "pipelined grid<=2048", 13: "pipelined unroll1 grid<=1024", 14: "pipelined block256 grid<=2048"}


def main():
    sizes = [64, 256, 1024, 4096, 16384, 65536, 262144]
    variants = [0]
    if "--variants" in sys.argv:  # the ring-chunk regime per kernel variant
        sizes, variants = [4096, 16384, 65536], [0, 9, 10, 11, 12, 13, 14]
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    pool_a = torch.empty(FOOT // 4, device=dev).uniform_(-1, 1)
    pool_b = torch.empty(FOOT // 4, device=dev).uniform_(-1, 1)
    for kib, var in [(k, v) for k in sizes for v in variants]:
        hip.set_variant(var)
        nbytes = kib << 10
        n = nbytes // 4
        slots = max(2, FOOT // nbytes)
        pa = [pool_a.data_ptr() + i * nbytes for i in range(slots)]
        pb = [pool_b.data_ptr() + i * nbytes for i in range(slots)]
        k = max(40, min(2000, (256 << 20) // nbytes * 20))
        for i in range(min(k, 20)):
            hip.reduce_ptr("sum", "f32", pa[i % slots], pb[i % slots], n, s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(k):
            hip.reduce_ptr("sum", "f32", pa[i % slots], pb[i % slots], n, s)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / k
        alg = 3 * nbytes
        print(json.dumps({"chunk_kib": kib, "variant": var, "name": VARIANTS[var], "launches": k, "slots": slots, "us_per_launch": round(us, 3),
                          "alg_GBs": round(alg / (us / 1e6) / 1e9, 1),
                          "frac_of_8TBs": round(alg / (us / 1e6) / 8e12, 4)}), flush=True)
    hip.set_variant(0)


if __name__ == "__main__":
    main()
