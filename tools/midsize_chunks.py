"""MEASUREMENT: what the ring routes lose to per-launch ramp and drain
(VERDICT r5 #6).

The reference ring route reduces 2(P - 1) chunks per allreduce, one launch
each (AllreduceRingChunked at P = 8 and 256 MiB per rank: 14 launches of
16 MiB, gloo/allreduce_ring_chunked.h:106-158).  A multi-range launch would
pay one ramp and drain for several chunks.  This measures the upper bound of
that saving on one MI355X with the product kernel (gloo_hip_reduce, fp32
sum, in place, 2 reads + 1 write per element):

  separate  K back-to-back launches of c bytes each (distinct buffers, so no
            launch reads what the previous one wrote from the Infinity Cache)
  one       ONE launch over K * c bytes (the same bytes)

HIP events on the launch stream around each variant, median of `reps`.  One
JSON line per chunk size: microseconds, the launch-rate fraction of 8 TB/s
for each, and separate/one (the ramp-and-drain overhead a merged launch
would remove).  Usage: python tools/midsize_chunks.py [K] [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import gloo_amd as hip
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 14
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = torch.cuda.current_stream(dev)
    for mib in (1, 4, 16, 64):
        n = mib * (1 << 20) // 4
        dst = torch.empty(K * n, dtype=torch.float32, device=dev).uniform_(-1, 1)
        src = torch.empty(K * n, dtype=torch.float32, device=dev).uniform_(-1, 1)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

        def separate():
            for k in range(K):
                hip.reduce_ptr("sum", "f32", dst.data_ptr() + 4 * k * n, src.data_ptr() + 4 * k * n, n, s.cuda_stream)

        def one():
            hip.reduce_ptr("sum", "f32", dst.data_ptr(), src.data_ptr(), K * n, s.cuda_stream)

        out = {"chunk_mib": mib, "K": K}
        for name, fn in (("separate", separate), ("one", one)):
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                ev[0].record(s)
                fn()
                ev[1].record(s)
                ev[1].synchronize()
                ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
            ts.sort()
            us = ts[len(ts) // 2]
            out[name + "_us"] = round(us, 2)
            out[name + "_frac_of_8TBs"] = round(3 * 4 * K * n / (us * 1e-6) / 8e12, 4)
        out["separate_over_one"] = round(out["separate_us"] / out["one_us"], 4)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
