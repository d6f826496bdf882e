"""Host-staged chunk reduction: the staging choices of gloo_hip_reduce_staged
timed interleaved, several rounds, so box-to-box PCIe spread does not decide
the default piece size (BENCH_r05 read 16 MiB pieces at 62.5
GiB/s, the round-6 final tree's bench 54.3).

Each round times, in turn, on one 64 MiB fp32 chunk in pinned host memory:
  serial      torch H2D dst + H2D src + kernel + D2H dst on one stream
  one_pass    gloo_hip_reduce_staged with the whole chunk as one piece
  pieces_16   the library's pipeline in 16 MiB pieces (its minimum)
  pieces_32   ... in 32 MiB pieces
  zero_copy   piece 0: the kernel reads and writes the mapped host buffers
Each figure is the mean of `iters` back-to-back calls; every variant's result
is checked against the IEEE sum once.  One JSON line per (round, variant),
then one summary line with the per-variant medians.

  python tools/host_staged_sweep.py [--rounds 7] [--iters 20] [--mib 64]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--mib", type=int, default=64)
    args = ap.parse_args()

    import torch
    import gloo_amd as hip

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n = args.mib * (1 << 20) // 4
    h_dst = torch.empty(n, dtype=torch.float32, pin_memory=True).uniform_(-1, 1)
    h_src = torch.empty(n, dtype=torch.float32, pin_memory=True).uniform_(-1, 1)
    d_dst = torch.empty(n, dtype=torch.float32, device=dev)
    d_src = torch.empty(n, dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream(dev)

    def serial():
        d_dst.copy_(h_dst, non_blocking=True)
        d_src.copy_(h_src, non_blocking=True)
        hip.reduce_ptr("sum", "f32", d_dst.data_ptr(), d_src.data_ptr(), n, s.cuda_stream)
        h_dst.copy_(d_dst, non_blocking=True)

    def staged(piece):
        return lambda: hip.reduce_staged("sum", "f32", h_dst.data_ptr(), h_src.data_ptr(), n, d_dst.data_ptr(),
                                         d_src.data_ptr(), piece, s.cuda_stream)

    variants = [("serial", serial), ("one_pass", staged(n)), ("pieces_16", staged((16 << 20) // 4)),
                ("pieces_32", staged((32 << 20) // 4)), ("zero_copy", staged(0))]

    # every variant gives the IEEE sum on the host
    a0 = torch.empty(n, dtype=torch.float32).uniform_(-1, 1)
    want = a0 + h_src
    verified = {}
    for name, fn in variants:
        h_dst.copy_(a0)
        fn()
        torch.cuda.synchronize(dev)
        verified[name] = bool(torch.equal(h_dst, want))

    def timed(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.iters):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / args.iters

    per = {name: [] for name, _ in variants}
    for r in range(args.rounds):
        for name, fn in variants:
            dt = timed(fn)
            gbs = 3.0 * n * 4 / dt / GIB
            per[name].append(gbs)
            print(json.dumps({"round": r, "variant": name, "ms_per_chunk": round(dt * 1e3, 3),
                              "gib_s_alg": round(gbs, 2)}), flush=True)
    print(json.dumps({"summary": True, "chunk_mib": args.mib, "rounds": args.rounds, "iters": args.iters,
                      "median_gib_s_alg": {k: round(statistics.median(v), 2) for k, v in per.items()},
                      "min_gib_s_alg": {k: round(min(v), 2) for k, v in per.items()},
                      "max_gib_s_alg": {k: round(max(v), 2) for k, v in per.items()},
                      "verified": verified}), flush=True)
    if not all(verified.values()):
        sys.exit(1)


if __name__ == "__main__":
    main()
