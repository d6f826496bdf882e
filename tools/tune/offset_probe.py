#!/usr/bin/env python3
"""MEASUREMENT ONLY: does the relative placement of the two operands in HBM
change the config-2 kernel's rate?  In-place fp32 sum of 64 MiB chunks (the
product kernel, gloo_hip_reduce), six rotated (dst, src) pairs; each src sits
`off` bytes past a 2 MiB-aligned block (dst stays aligned), off in a sweep of
multiples of 256 B (no element misalignment).  300 back-to-back launches
between two events per offset, offsets alternated over 3 repetitions.
One JSON line per (rep, offset)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import gloo_amd as hip  # noqa: E402

N = 16 << 20
OFFS = [0, 256, 4096, 8192, 65536, 1 << 20, (1 << 20) + 4096]


def main():
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    dsts = [torch.rand(N, device=dev) for _ in range(6)]
    # one oversized block per pair, src carved at each offset
    srcblk = [torch.rand(N + (4 << 20) // 4, device=dev) for _ in range(6)]
    for rep in range(3):
        for off in OFFS:
            srcs = [b.data_ptr() + ((-b.data_ptr()) % (2 << 20)) + off for b in srcblk]
            for i in range(12):
                hip.reduce_ptr("sum", "f32", dsts[i % 6].data_ptr(), srcs[i % 6], N, s)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(300):
                hip.reduce_ptr("sum", "f32", dsts[i % 6].data_ptr(), srcs[i % 6], N, s)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 300
            print(json.dumps({"rep": rep, "src_offset": off, "dst_mod_2MiB": dsts[0].data_ptr() % (2 << 20),
                              "us": round(us, 3), "frac_of_8TBs": round(3 * N * 4 / (us / 1e6) / 8e12, 4)}),
                  flush=True)


if __name__ == "__main__":
    main()
