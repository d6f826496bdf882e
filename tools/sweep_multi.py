#!/usr/bin/env python3
"""Local multi-pointer fold (rows a9/a13: AllreduceLocal / CudaLocalNativeReduce,
gloo/allreduce_local.cc:28-33) at 64 MiB fp32 per source, k = 2..8 sources.

Two ways to compute dst = s0 + s1 + ... + s(k-1) with the same left-fold bits:
  fused:    one gloo_hip_reduce_multi launch, (k+1)*n*4 algorithmic bytes
  pairwise: the reference's loop, k-1 in-place gloo_hip_reduce calls, 3*(k-1)*n*4 bytes
Times are HIP events on the launching stream over back-to-back launches; two
rotated source sets keep the footprint above the 256 MiB Infinity Cache.
One JSON line per k.  Bits: fused == pairwise is asserted for every k."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import gloo_amd as hip  # noqa: E402

N = 16 << 20  # fp32 elements = 64 MiB per source
PEAK = 8e12


def main():
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=dev).manual_seed(3)
    sets = [[torch.rand(N, device=dev, generator=g) * 2 - 1 for _ in range(8)] for _ in range(2)]
    dsts = [torch.empty(N, device=dev) for _ in range(2)]
    ks = range(2, 9)
    if "--k" in sys.argv:  # one k only (PMC passes)
        ks = [int(sys.argv[sys.argv.index("--k") + 1])]
    for k in ks:
        # bits first: the fused left fold equals the reference's pairwise loop
        ref = sets[0][0].clone()
        for j in range(1, k):
            hip.reduce_ptr("sum", "f32", ref.data_ptr(), sets[0][j].data_ptr(), N, s)
        hip.reduce_multi_ptr("sum", "f32", dsts[0].data_ptr(), [t.data_ptr() for t in sets[0][:k]], N, s)
        torch.cuda.synchronize()
        assert torch.equal(ref.view(torch.int32), dsts[0].view(torch.int32)), f"k={k}: fused != pairwise"

        def fused(i):
            hip.reduce_multi_ptr("sum", "f32", dsts[i % 2].data_ptr(),
                                 [t.data_ptr() for t in sets[i % 2][:k]], N, s)

        def pairwise(i):
            src = sets[i % 2]
            d = dsts[i % 2]
            hip.reduce3_ptr("sum", "f32", d.data_ptr(), src[0].data_ptr(), src[1].data_ptr(), N, s)
            for j in range(2, k):
                hip.reduce_ptr("sum", "f32", d.data_ptr(), src[j].data_ptr(), N, s)

        out = {"k": k, "n": N, "dtype": "f32"}
        for name, fn, nbytes in (("fused", fused, (k + 1) * N * 4), ("pairwise", pairwise, 3 * (k - 1) * N * 4)):
            for i in range(4):
                fn(i)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            steps = 60
            e0.record()
            for i in range(steps):
                fn(i)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / steps
            out[name] = {"us": round(us, 2), "alg_bytes": nbytes,
                         "GBs": round(nbytes / (us / 1e6) / 1e9, 1),
                         "frac_of_8TBs": round(nbytes / (us / 1e6) / PEAK, 4)}
        out["speedup_fused"] = round(out["pairwise"]["us"] / out["fused"]["us"], 2)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
