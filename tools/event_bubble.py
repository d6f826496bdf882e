#!/usr/bin/env python3
"""Where does the K = 20 event region lose time against K = 1000?

Measures the config-2 kernel (64 MiB fp32 in-place sum, 6 rotated pairs) on
one stream with HIP events placed several ways:
  ends_k{K}      events after launch 1 and after launch K (bench.py's region),
                 the GPU idle (synchronised) before launch 1;
  before_k{K}    an event before launch 1 and after launch K, region / K;
  every          an event after every launch of a long run: each interval
                 is one launch-to-launch time, so a marker between two
                 kernels shows up as a longer interval, and the first
                 intervals after an idle GPU show any start-up transient.
One JSON line per measurement.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import gloo_amd as hip

    dev = torch.device("cuda:0")
    n = 64 * (1 << 20) // 4
    g = torch.Generator(device=dev).manual_seed(7)
    pairs = [(torch.rand(n, device=dev, generator=g), torch.rand(n, device=dev, generator=g)) for _ in range(6)]
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    def step(i):
        d, s = pairs[i % len(pairs)]
        hip.reduce_ptr("sum", "f32", d.data_ptr(), s.data_ptr(), n, sh)

    def ev():
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        return e

    for i in range(50):
        step(i)
    torch.cuda.synchronize(dev)

    def out(**kw):
        print(json.dumps(kw), flush=True)

    import ctypes
    rt = ctypes.CDLL("libamdhip64.so.7")   # the runtime torch already loaded (same soname)

    class RawEv:
        """hipEventCreateWithFlags(flags) / hipEventRecord / hipEventElapsedTime."""
        def __init__(self, flags):
            self.h = ctypes.c_void_p()
            assert rt.hipEventCreateWithFlags(ctypes.byref(self.h), ctypes.c_uint(flags)) == 0

        def record(self):
            assert rt.hipEventRecord(self.h, ctypes.c_void_p(sh)) == 0
            return self

        def ms_to(self, other):
            ms = ctypes.c_float()
            assert rt.hipEventElapsedTime(ctypes.byref(ms), self.h, other.h) == 0
            return ms.value

    flag_sets = {"dev": 0x40000000, "nofence": 0x20000000, "default": 0x0}

    for rep in range(5):
        for fname, fl in flag_sets.items():
            for K in (20, 1000):
                torch.cuda.synchronize(dev)
                step(0)
                r0 = RawEv(fl).record()
                for i in range(1, K):
                    step(i)
                r1 = RawEv(fl).record()
                torch.cuda.synchronize(dev)
                out(kind=f"raw_{fname}_ends_k{K}", rep=rep, us=round(r0.ms_to(r1) * 1e3 / (K - 1), 3))
            torch.cuda.synchronize(dev)
            evs = []
            for i in range(100):
                step(i)
                evs.append(RawEv(fl).record())
            torch.cuda.synchronize(dev)
            iv = [evs[i].ms_to(evs[i + 1]) * 1e3 for i in range(len(evs) - 1)]
            out(kind=f"raw_{fname}_every", rep=rep, mean=round(sum(iv[10:]) / len(iv[10:]), 3))

        for K in (20, 100, 1000):
            torch.cuda.synchronize(dev)
            step(0)
            e0 = ev()
            for i in range(1, K):
                step(i)
            e1 = ev()
            torch.cuda.synchronize(dev)
            out(kind=f"ends_k{K}", rep=rep, us=round(e0.elapsed_time(e1) * 1e3 / (K - 1), 3))

            torch.cuda.synchronize(dev)
            e0 = ev()
            for i in range(K):
                step(i)
            e1 = ev()
            torch.cuda.synchronize(dev)
            out(kind=f"before_k{K}", rep=rep, us=round(e0.elapsed_time(e1) * 1e3 / K, 3))

        for K in (20, 1000):
            # hipExtLaunchKernel events bound to launch 1's start and launch K's end
            x0 = torch.cuda.Event(enable_timing=True)
            x1 = torch.cuda.Event(enable_timing=True)
            x0.record(stream)
            x1.record(stream)
            torch.cuda.synchronize(dev)
            hip.set_launch_events(x0, None)
            step(0)
            for i in range(1, K - 1):
                step(i)
            hip.set_launch_events(None, x1)
            step(K - 1)
            torch.cuda.synchronize(dev)
            out(kind=f"ext_k{K}", rep=rep, us=round(x0.elapsed_time(x1) * 1e3 / K, 3))

        torch.cuda.synchronize(dev)
        evs = []
        for i in range(200):
            step(i)
            evs.append(ev())
        torch.cuda.synchronize(dev)
        iv = [evs[i].elapsed_time(evs[i + 1]) * 1e3 for i in range(len(evs) - 1)]
        out(kind="every", rep=rep, first10=[round(x, 2) for x in iv[:10]],
            mean_1_19=round(sum(iv[:19]) / 19, 3), mean_rest=round(sum(iv[19:]) / len(iv[19:]), 3))


if __name__ == "__main__":
    main()
