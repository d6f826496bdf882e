"""Where the driver-shaped bench's wall time goes beyond its kernels (K = 20).

bench.py's value is K launches' algorithmic bytes over the host wall time of
the bracket [sync, K launches, spin on the last event, sync]; its roofline
figure is the launch-to-launch time of launches 2..K from HIP events.  At
K = 20 the wall per step runs ~2 us above the event figure.  This tool
repeats the bench's timed region and splits its host time: the first
launch's enqueue, the other enqueues, the wait for the end (spin), the closing
synchronize; and on the GPU clock, launch 1 (an extra event before it) against
launches 2..K.  One JSON line per repetition, then medians.

  python tools/bench_overhead.py [--reps 15] [--steps 20]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bench import HipEvent  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import torch
    import gloo_amd as hip

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n = 64 * (1 << 20) // 4
    g = torch.Generator(device=dev).manual_seed(1234)
    pairs = [(torch.rand(n, device=dev, generator=g) * 2 - 1, torch.rand(n, device=dev, generator=g) * 2 - 1)
             for _ in range(6)]
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    def step(i):
        d, s = pairs[i % len(pairs)]
        hip.reduce_ptr("sum", "f32", d.data_ptr(), s.data_ptr(), n, sh)

    for i in range(5):
        step(i)
    torch.cuda.synchronize(dev)
    rows = []
    for rep in range(args.reps):
        e_pre, e_start, e_end = HipEvent(stream), HipEvent(stream), HipEvent(stream)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        e_pre.record()
        t1 = time.perf_counter()
        step(0)
        t2 = time.perf_counter()
        e_start.record()
        for i in range(1, args.steps):
            step(i)
        e_end.record()
        t3 = time.perf_counter()
        e_end.spin()
        t4 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t5 = time.perf_counter()
        first_ms = e_pre.elapsed_ms(e_start)
        rest_ms = e_start.elapsed_ms(e_end)
        row = {"rep": rep, "wall_us": round((t5 - t0) * 1e6, 1), "pre_record_us": round((t1 - t0) * 1e6, 1),
               "launch1_enqueue_us": round((t2 - t1) * 1e6, 1), "enqueue_rest_us": round((t3 - t2) * 1e6, 1),
               "spin_us": round((t4 - t3) * 1e6, 1), "sync_us": round((t5 - t4) * 1e6, 1),
               "gpu_launch1_us": round(first_ms * 1e3, 2),
               "gpu_launch_avg_2_to_k_us": round(rest_ms * 1e3 / (args.steps - 1), 3),
               "wall_minus_gpu_us": round((t5 - t0) * 1e6 - (first_ms + rest_ms) * 1e3, 1)}
        rows.append(row)
        print(json.dumps(row), flush=True)
        for e in (e_pre, e_start, e_end):
            e.destroy()
    med = {k: statistics.median(r[k] for r in rows) for k in rows[0] if k != "rep"}
    print(json.dumps({"summary": True, "steps": args.steps, "median": med}), flush=True)


if __name__ == "__main__":
    main()
