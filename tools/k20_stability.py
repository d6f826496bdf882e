#!/usr/bin/env python3
"""Spread of the bench's K = 20 kernel average, and whether a longer GPU
pre-warm before the W = 5 warmup steps changes it.

Each trial idles the GPU for `--idle-ms`, optionally streams 1 GiB copies for
`prewarm` ms, runs W warmup launches, then times K back-to-back launches the
way bench.py does (events after launch 1 and after launch K).  Trials
alternate the pre-warm settings so slow drift hits them alike.  One JSON line
per trial.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--trials", type=int, default=8)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--prewarm-ms", default="0,20,200")
    p.add_argument("--idle-ms", type=float, default=300.0)
    args = p.parse_args()

    import torch
    import gloo_amd as hip

    dev = torch.device("cuda:0")
    n = 64 * (1 << 20) // 4
    g = torch.Generator(device=dev).manual_seed(1234)
    pairs = [(torch.rand(n, device=dev, generator=g) * 2 - 1, torch.rand(n, device=dev, generator=g) * 2 - 1)
             for _ in range(6)]
    big_a = torch.empty(1 << 28, dtype=torch.float32, device=dev)
    big_b = torch.empty_like(big_a)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    def step(i):
        d, s = pairs[i % len(pairs)]
        hip.reduce_ptr("sum", "f32", d.data_ptr(), s.data_ptr(), n, sh)

    def prewarm(ms):
        t_end = time.perf_counter() + ms / 1e3
        while time.perf_counter() < t_end:
            big_b.copy_(big_a)
            torch.cuda.synchronize(dev)

    settings = [float(x) for x in args.prewarm_ms.split(",")]
    for t in range(args.trials):
        for pw in settings:
            torch.cuda.synchronize(dev)
            time.sleep(args.idle_ms / 1e3)
            prewarm(pw)
            for i in range(args.warmup):
                step(i)
            torch.cuda.synchronize(dev)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            step(0)
            e0.record(stream)
            for i in range(1, args.steps):
                step(i)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            us = e0.elapsed_time(e1) * 1e3 / (args.steps - 1)
            print(json.dumps({"trial": t, "prewarm_ms": pw, "kernel_us": round(us, 3),
                              "frac": round(3 * n * 4 / (us * 1e-6) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
