#!/usr/bin/env python3
"""Collectives benchmark: BASELINE.json configs 1, 3, 4, 5.

  config 1  reference AllreduceRingChunked<float>, size=2, TCP loopback, CPU
            (oracle/_ref, built from /root/reference) — the plumbing baseline
  config 3  ring-chunked fp32 sum, P ranks, 256 MiB per rank, chunks moved
            GPU->GPU (xGMI when ranks sit on different GPUs)
  config 4  halving-doubling fp32 sum, P ranks, sizes 1 KiB .. 1 GiB (--algo4 bcube
            --base B: AllreduceBcube instead, the reference benchmark's
            `allreduce_bcube --base`, gloo/benchmark/options.cc:80)
  config 5  reduce-scatter HD, fp16 / bf16, sum / product / min / max

Ranks are threads of this process, rank r on GPU r % device_count (on a
1-GPU box every rank shares the GPU: the data path is then HBM->HBM copies,
not xGMI — the JSON says which).  Per run: wall time (slowest rank), and with
profiling the reduce-kernel time of every chunk reduction (HIP events), so the
per-GPU reduce GiB/s inside a live collective is reported next to the
end-to-end rate.  One JSON line per measurement.
"""
import argparse
import json
import os
import sys
import threading
import time
import uuid

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)


def run_collective(torch, algo, op, dtype, P, n, iters, profile=True, recv=None):
    import gloo_amd
    ndev = torch.cuda.device_count()
    es = gloo_amd.dtype_size(dtype)
    bufs = []
    for r in range(P):
        d = torch.device("cuda", r % ndev)
        bufs.append(torch.ones(n * es // 4 if es >= 4 else (n * es + 3) // 4, dtype=torch.float32, device=d)
                    if dtype == "f32" else torch.zeros(n * es, dtype=torch.uint8, device=d))
    torch.cuda.synchronize()
    url = "mem:" + uuid.uuid4().hex
    times = [[] for _ in range(P)]
    stats = [None] * P
    errors = []
    bar = threading.Barrier(P)

    def body(r):
        try:
            dev = r % ndev
            torch.cuda.set_device(dev)
            ctx = gloo_amd.Context(r, P, url, device=dev, timeout_ms=120000)
            a = gloo_amd.Algorithm(ctx, algo, op, dtype, [bufs[r].data_ptr()], n, recv_elems=recv)
            a.set_profiling(profile)
            a.run()  # warmup
            acc = {"reduce_s": 0.0, "reduce_bytes": 0.0, "reductions": 0, "wait_s": 0.0}
            for _ in range(iters):
                bar.wait()
                t0 = time.perf_counter()
                a.run()
                times[r].append(time.perf_counter() - t0)
                st = a.stats()
                for k in acc:
                    acc[k] += st[k]
            stats[r] = acc
            bar.wait()
            a.close()
            ctx.close()
        except Exception as e:  # noqa: BLE001
            errors.append((r, repr(e)))
            bar.abort()

    ts = [threading.Thread(target=body, args=(r,)) for r in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errors:
        raise RuntimeError(errors)
    per_iter = [max(times[r][i] for r in range(P)) for i in range(iters)]
    per_iter.sort()
    return per_iter, stats


def run_collective_procs(torch, dist, algo, op, dtype, P, n, iters, store, profile=True, recv=None):
    """Same measurement with THIS process as one rank (torch.distributed.run
    launch); timings gathered over torch.distributed's gloo backend."""
    import gloo_amd
    rank = dist.get_rank()
    ndev = torch.cuda.device_count()
    dev = rank % ndev
    torch.cuda.set_device(dev)
    es = gloo_amd.dtype_size(dtype)
    buf = torch.zeros(max(4, n * es), dtype=torch.uint8, device=f"cuda:{dev}")
    if dtype == "f32":
        buf.view(torch.float32)[:n].fill_(1.0)
    torch.cuda.synchronize()
    ctx = gloo_amd.Context(rank, P, store, device=dev, timeout_ms=120000)
    a = gloo_amd.Algorithm(ctx, algo, op, dtype, [buf.data_ptr()], n, recv_elems=recv)
    a.set_profiling(profile)
    a.run()
    times, acc = [], {"reduce_s": 0.0, "reduce_bytes": 0.0, "reductions": 0, "wait_s": 0.0}
    for _ in range(iters):
        dist.barrier()
        t0 = time.perf_counter()
        a.run()
        times.append(time.perf_counter() - t0)
        st = a.stats()
        for k in acc:
            acc[k] += st[k]
    a.close()
    ctx.close()
    allt = [None] * P
    alls = [None] * P
    dist.all_gather_object(allt, times)
    dist.all_gather_object(alls, acc)
    per_iter = sorted(max(allt[r][i] for r in range(P)) for i in range(iters))
    return per_iter, alls


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--ranks", type=int, default=8)
    p.add_argument("--configs", default="1,3,4,5")
    p.add_argument("--iters", type=int, default=5)
    p.add_argument("--max-lg", type=int, default=30, help="config 4: largest size, log2 bytes per rank")
    p.add_argument("--algo4", default="halving_doubling", choices=["halving_doubling", "bcube"])
    p.add_argument("--base", type=int, default=2, help="--algo4 bcube: the group size (gloo::Context::base)")
    args = p.parse_args()
    cfgs = set(args.configs.split(","))
    import torch
    ndev = torch.cuda.device_count()
    P = args.ranks
    world = int(os.environ.get("WORLD_SIZE", "0"))
    emit = True
    if world:
        # ranks are processes: one per GPU (wrapping on a small box)
        import tempfile
        import torch.distributed as dist
        dist.init_process_group("gloo")
        P = world
        emit = dist.get_rank() == 0
        obj = [tempfile.mkdtemp(prefix="gloo_amd_coll_")] if emit else [None]
        dist.broadcast_object_list(obj, src=0)
        counter = [0]

        def run_collective(torch, algo, op, dtype, P, n, iters, profile=True, recv=None):  # noqa: F811
            counter[0] += 1
            return run_collective_procs(torch, dist, algo, op, dtype, P, n, iters,
                                        "file:%s/%d" % (obj[0], counter[0]), profile, recv)
    else:
        run_collective = globals()["run_collective"]
    layout = "processes" if world else "threads"
    where = ("xGMI peer copies" if ndev >= P else f"{P} ranks on {ndev} GPU(s): HBM-local copies") + \
        f", ranks as {layout}"
    import builtins
    _print = builtins.print

    def print(*a, **k):  # noqa: A001
        if emit:
            _print(*a, **k)
    if "1" in cfgs and emit:
        import ctypes
        import oracle
        if oracle.ref_available():
            L = oracle.ref()
            L.ref_allreduce_timed.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                              ctypes.POINTER(ctypes.c_double)]
            for n in (1 << 20, 1 << 24):
                sec = ctypes.c_double()
                rc = L.ref_allreduce_timed(0, 2, n, 5, ctypes.byref(sec))
                print(json.dumps({"config": 1, "impl": "reference CPU AllreduceRingChunked<float>",
                                  "ranks": 2, "transport": "tcp loopback (threads)", "elements": n,
                                  "rc": rc, "ms": round(sec.value * 1e3, 3),
                                  "payload_gib_s": round(n * 4 / sec.value / GIB, 3)}), flush=True)
    if "3" in cfgs:
        n = 64 << 20  # 256 MiB of fp32 per rank
        per, st = run_collective(torch, "ring_chunked", "sum", "f32", P, n, args.iters)
        t = per[len(per) // 2]
        red_s = max(s["reduce_s"] for s in st) / args.iters
        red_b = st[0]["reduce_bytes"] / args.iters
        print(json.dumps({"config": 3, "algo": "ring_chunked", "ranks": P, "gpus": ndev, "data_path": where,
                          "bytes_per_rank": n * 4, "ms_p50": round(t * 1e3, 3),
                          "algbw_gib_s": round(n * 4 / t / GIB, 2),
                          "busbw_gib_s": round(2 * (P - 1) / P * n * 4 / t / GIB, 2),
                          "reduce_kernel_gib_s_per_gpu": round(red_b / red_s / GIB, 1) if red_s else None,
                          "reduce_kernel_ms_per_run": round(red_s * 1e3, 3),
                          "host_wait_ms_per_run": round(max(s["wait_s"] for s in st) / args.iters * 1e3, 3)}),
              flush=True)
    if "4" in cfgs:
        for lg in range(10, args.max_lg + 1, 2):  # 1 KiB .. 1 GiB per rank
            n = max(1, (1 << lg) // 4)
            it = args.iters if lg < 28 else 3
            # latency: no profiling events, so the plan replays as a hipGraph
            recv4 = [args.base] if args.algo4 == "bcube" else None
            per, st = run_collective(torch, args.algo4, "sum", "f32", P, n, max(it, 3), profile=False, recv=recv4)
            print(json.dumps({"config": 4, "algo": args.algo4, "ranks": P, "gpus": ndev,
                              **({"base": args.base} if args.algo4 == "bcube" else {}),
                              "data_path": where, "bytes_per_rank": n * 4,
                              "env": {k: v for k, v in os.environ.items() if k.startswith("GLOO_AMD_")},
                              "us_p50": round(per[len(per) // 2] * 1e6, 1),
                              "us_max": round(per[-1] * 1e6, 1),
                              "busbw_gib_s": round(2 * (P - 1) / P * n * 4 / per[len(per) // 2] / GIB, 3)}),
                  flush=True)
    if "5" in cfgs:
        for dtype in ("f16", "bf16"):
            for op in ("sum", "product", "min", "max"):
                n = 16 << 20
                chunk = (n + P - 1) // P
                recv = [min(chunk, max(0, n - i * chunk)) for i in range(P)]
                per, st = run_collective(torch, "reduce_scatter", op, dtype, P, n, args.iters, recv=recv)
                red_s = max(s["reduce_s"] for s in st) / args.iters
                red_b = st[0]["reduce_bytes"] / args.iters
                print(json.dumps({"config": 5, "algo": "reduce_scatter_hd", "dtype": dtype, "op": op,
                                  "ranks": P, "gpus": ndev, "data_path": where, "elements_per_rank": n,
                                  "ms_p50": round(per[len(per) // 2] * 1e3, 3),
                                  "reduce_kernel_gib_s_per_gpu": round(red_b / red_s / GIB, 1) if red_s else None}),
                      flush=True)


if __name__ == "__main__":
    main()
