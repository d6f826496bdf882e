#!/usr/bin/env python3
"""Benchmark: device-resident per-chunk reduction (fp32 sum), Gloo hot path.

BASELINE.json metric "device-resident chunk-reduce GiB/s (fp32 sum) + % HBM
roofline, 1/2/4/8 GPU" on config 2: one 64 MiB fp32 chunk reduced in place
(dst += src, the form every schedule calls through ReductionFunction::call,
gloo/algorithm.h:75-77) by the HIP kernel behind include/gloo_amd.h.

One step = one kernel over one 64 MiB chunk.  Inputs are resident in HBM
before the timed region.  Six (dst, src) pairs are rotated (768 MiB footprint,
3x the 256 MiB Infinity Cache) so every step streams from HBM.

Multi-GPU: one process per GPU (torch.distributed.run), each GPU reduces its
own chunks — the reduction partitions into independent units, so there is no
data-path collective ("scaling": "weak"); torch.distributed's gloo backend is
used only for the harness barrier and the max-over-ranks time.

Also reported (rank 0, N=1 only): the reference's own gloo::sum<float>
(oracle/_ref, built from /root/reference as it ships) timed on the host cores
(`cpu_baseline`), and the host-staged rate of a chunk that starts and ends in
pinned host memory (H2D + kernel + D2H).
"""
import argparse
import contextlib
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident chunk-reduce GiB/s (fp32 sum) + % HBM roofline, 1/2/4/8 GPU"
WORKLOAD = ("single-GPU device-resident fp32 sum-reduce kernel, 64 MiB chunk "
            "(allreduce_local path, no transport)")
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
GIB = float(1 << 30)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--config3-variants", default="",
                   help="N>1: comma list of config-3 variants after the default (diagnosis)")
    p.add_argument("--config3-only", action="store_true",
                   help="N>1: stop the xGMI section after config 3 (diagnosis)")
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--chunk-mib", type=int, default=64)
    p.add_argument("--pairs", type=int, default=6, help="rotated (dst, src) pairs")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="bounded CPU-baseline sample (seconds of CPU work)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-config1", action="store_true", help="skip the config-1 CPU allreduce in cpu_baseline")
    p.add_argument("--config1-seconds", type=float, default=2.0,
                   help="config 1: minimum seconds per batch (gloo/benchmark default 2 s)")
    p.add_argument("--no-host-staged", action="store_true")
    p.add_argument("--variant", type=int, default=0, help="kernel variant (tuning)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    p.add_argument("--no-allreduce", action="store_true",
                   help="N>1: skip the config-3 xGMI ring-chunked allreduce section")
    p.add_argument("--allreduce-mib", type=int, default=256, help="config 3: MiB per rank")
    p.add_argument("--allreduce-iters", type=int, default=5)
    p.add_argument("--sweep-seconds", type=float, default=0.2,
                   help="N>1 config-4 sweep: minimum seconds per timed batch (gloo/benchmark default 2 s)")
    p.add_argument("--quick", action="store_true",
                   help="N>1: config 3 + one variant, short HD sweep, RS at 16 Mi (rehearsals)")
    p.add_argument("--watchdog-seconds", type=float, default=180.0,
                   help="N>1: the xGMI section may go this long without progress (a hang); then the line is "
                        "printed and the job exits 3")
    p.add_argument("--watchdog-total-seconds", type=float, default=1500.0,
                   help="N>1: the xGMI section's overall limit (same outcome)")
    return p.parse_args()


def relaunch_distributed(args):
    """`python bench.py --gpus N` outside torch.distributed.run: start the
    launcher as a child process (no exec) before anything touches the GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(29500 + os.getpid() % 1000), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


_LAST_PROGRESS = [time.time()]


def progress(msg):
    """One progress line on stderr (every rank): a long multi-rank run keeps
    writing, and a stuck section names itself.  Also the watchdog's clock."""
    _LAST_PROGRESS[0] = time.time()
    print(f"[bench r{os.environ.get('RANK', '0')} {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def host_cores():
    """(cores, how): the CPU share this process may use — the cgroup quota
    (/sys/fs/cgroup/cpu.max) when one is set, else the affinity mask."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            return max(1, int(int(quota) / int(period))), f"cgroup quota {quota}/{period} (/sys/fs/cgroup/cpu.max)"
    except (OSError, ValueError):
        pass
    try:
        n = len(os.sched_getaffinity(0))
        return n, "sched_getaffinity (no cgroup CPU quota)"
    except AttributeError:
        return os.cpu_count() or 1, "os.cpu_count"


def cpu_baseline(args, n):
    """The reference's gloo::sum<float> on host memory (64 MiB chunks, the
    same rotation as the GPU leg), bounded to ~args.cpu_seconds of CPU work:
    the 2-operand in-place form (how ReductionFunction<T>::sum calls it) and
    the 3-operand form, on 1 thread (how Gloo calls it) and split over the
    box's CPU share; plus BASELINE config 1 — the reference's own
    AllreduceRingChunked<float>, 2 ranks over TCP loopback — with the
    reference benchmark's methodology (gloo/benchmark/runner.cc:311-363)."""
    import numpy as np
    import oracle
    if oracle.ref_available():
        L = oracle.ref_baseline()
        f3 = L.ref_base_sum_f32
        f2 = L.ref_base_sum2_f32
        kind = "reference"
    else:
        f3 = oracle.lib().oracle_sum_f32_mt
        f2 = lambda a, b, m, t: f3(a, a, b, m, t)  # noqa: E731
        kind = "port"
    pairs = max(2, args.pairs // 2)
    rng = np.random.default_rng(1)
    bufs = [(rng.uniform(-1, 1, n).astype(np.float32), rng.uniform(-1, 1, n).astype(np.float32))
            for _ in range(pairs)]
    outs = [np.empty(n, np.float32) for _ in range(pairs)]

    def timed(form, threads, budget):
        done, t0 = 0, time.perf_counter()
        while True:
            d, s = bufs[done % pairs]
            if form == 2:
                f2(d.ctypes.data, s.ctypes.data, n, threads)
            else:
                f3(outs[done % pairs].ctypes.data, d.ctypes.data, s.ctypes.data, n, threads)
            done += 1
            el = time.perf_counter() - t0
            if el >= budget and done >= 3:
                return done, el

    for i in range(pairs):  # page in
        d, s = bufs[i]
        f3(outs[i].ctypes.data, d.ctypes.data, s.ctypes.data, n, 1)
    alg = 3.0 * n * 4
    nt, how = host_cores()
    nt = max(1, min(nt, os.cpu_count() or 1))
    res = {}
    for form, budget1 in ((2, args.cpu_seconds * 0.6), (3, args.cpu_seconds * 0.4)):
        c1, t1 = timed(form, 1, budget1)
        cn, tn = timed(form, nt, max(1.0, args.cpu_seconds / 5))
        res[form] = (round(alg * c1 / t1 / GIB, 3), c1, t1, round(alg * cn / tn / GIB, 3), cn, tn)
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "")
    except OSError:
        pass
    v2, v3 = res[2], res[3]
    out = {
        "value": v2[0], "unit": "GiB/s", "cores": 1, "kind": kind,
        "sample": (f"{v2[1]} calls of gloo::sum<float>(a,b,n) (the in-place 2-operand form, "
                   f"gloo/math.h:25-28), n={n} (64 MiB), {pairs} rotated pairs, {v2[2]:.1f} s, 1 thread as "
                   f"Gloo calls it; algorithmic bytes 3*n*4"),
        "three_operand": {"value": v3[0], "sample": f"{v3[1]} calls of gloo::sum<float>(c,a,b,n), c distinct, "
                                                    f"1 thread, {v3[2]:.1f} s"},
        "all_cores": {"value": v2[3], "threads": nt, "threads_from": how,
                      "three_operand_value": v3[3],
                      "sample": (f"{v2[4]} (2-operand) + {v3[4]} (3-operand) calls, range split over {nt} "
                                 f"std::threads, {v2[5]:.1f} + {v3[5]:.1f} s")},
        "cpu_model": model, "host_cpus_visible": os.cpu_count(),
    }
    if kind == "reference" and not args.no_config1:
        out["config1_allreduce_ring_chunked"] = config1(oracle, args)
    return out


@contextlib.contextmanager
def stdout_fd_to_stderr():
    """Gloo's TCP context prints its connectivity line with std::cout
    (gloo/transport/tcp/context.cc:243-246; the reference built here for
    config 1, and PyTorch's bundled copy behind init_process_group("gloo"));
    send fd 1 to stderr meanwhile so stdout carries only the bench's JSON
    line."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        os.dup2(saved, 1)
        os.close(saved)


def config1(oracle, args, n=1 << 24):
    """BASELINE config 1: the reference's AllreduceRingChunked<float>, size=2,
    2 ranks (threads) over TCP loopback, n = 16 Mi fp32; 5 warmup runs, then
    batches of runs until one lasts >= args.config1_seconds; p50 / p99 of the
    per-iteration latencies and the payload GiB/s n*4/p50
    (gloo/benchmark/runner.cc:311-363, :497-506)."""
    import numpy as np
    cap = 100000
    buf = (ctypes.c_double * cap)()
    cnt = ctypes.c_int(0)
    t0 = time.perf_counter()
    with stdout_fd_to_stderr():
        rc = oracle.ref().ref_allreduce_samples(0, 2, n, 5, args.config1_seconds, buf, cap, ctypes.byref(cnt))
    if rc:
        return {"error": oracle.ref().ref_last_error().decode()}
    s = np.sort(np.array(buf[:cnt.value]))
    p50, p99 = float(s[len(s) // 2]), float(s[min(len(s) - 1, int(len(s) * 0.99))])
    return {"elements": n, "ranks": 2, "transport": "tcp loopback (reference)", "samples": int(cnt.value),
            "p50_ms": round(p50 * 1e3, 3), "p99_ms": round(p99 * 1e3, 3),
            "payload_gib_s_p50": round(n * 4 / p50 / GIB, 3), "wall_s": round(time.perf_counter() - t0, 1)}


def host_staged(torch, hip, n, dev, iters=20):
    """Chunks starting and ending in pinned host memory (a transport recv
    buffer on a socket/NIC).  Ways to reduce them on the GPU:
      serial     H2D dst + H2D src + kernel + D2H dst, one stream;
      library_staged  gloo_hip_reduce_staged staging through device scratch
                 in its default 16 MiB pieces (a requested piece below
                 16 MiB is raised to it): H2D of piece k+1, the kernel of
                 piece k and D2H of piece k-1 overlap;
      library_staged_32MiB  the same in 32 MiB pieces;
      library_one_pass  the same with one piece (the chunk): serial through
                 the library;
      zero_copy_src  the accumulator stays in HBM and the kernel reads the
                 host chunk in place (the HOST-workspace allreduce's reduce);
      zero_copy_both the kernel reads both operands from host memory and
                 writes the result back there;
      library_default gloo_hip_reduce_staged with piece 0: zero-copy when both
                 host buffers are mapped (they are here), else 16 MiB pieces.
    GiB/s is algorithmic (3 * n * 4 B per reduction)."""
    import ctypes
    h_dst = torch.empty(n, dtype=torch.float32, pin_memory=True).uniform_(-1, 1)
    h_src = torch.empty(n, dtype=torch.float32, pin_memory=True).uniform_(-1, 1)
    d_dst = torch.empty(n, dtype=torch.float32, device=dev)
    d_src = torch.empty(n, dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream(dev)
    hiprt = ctypes.CDLL("libamdhip64.so")

    def devptr(t):
        p = ctypes.c_void_p()
        rc = hiprt.hipHostGetDevicePointer(ctypes.byref(p), ctypes.c_void_p(t.data_ptr()), 0)
        assert rc == 0, rc
        return p.value

    def timed(once, k=iters):
        for _ in range(2):
            once()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(k):
            once()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / k

    def serial():
        d_dst.copy_(h_dst, non_blocking=True)
        d_src.copy_(h_src, non_blocking=True)
        hip.reduce_ptr("sum", "f32", d_dst.data_ptr(), d_src.data_ptr(), n, s.cuda_stream)
        h_dst.copy_(d_dst, non_blocking=True)

    def staged(piece):
        # gloo_hip_reduce_staged: piece > 0 stages through the device
        # scratch; piece 0 is zero-copy on mapped buffers
        return lambda: hip.reduce_staged("sum", "f32", h_dst.data_ptr(), h_src.data_ptr(), n, d_dst.data_ptr(),
                                         d_src.data_ptr(), piece, s.cuda_stream)

    hs, hd = devptr(h_src), devptr(h_dst)

    def zc_src():
        hip.reduce_ptr("sum", "f32", d_dst.data_ptr(), hs, n, s.cuda_stream)

    def zc_both():
        hip.reduce_ptr("sum", "f32", hd, hs, n, s.cuda_stream)

    out = {}
    for name, fn in (("serial", serial), ("library_staged", staged(1)),
                     ("library_staged_32MiB", staged((32 << 20) // 4)), ("library_one_pass", staged(n)),
                     ("zero_copy_src", zc_src), ("zero_copy_both", zc_both),
                     ("library_default", staged(0))):
        dt = timed(fn)
        out[name] = {"gib_s_alg": round(3.0 * n * 4 / dt / GIB, 2), "ms_per_chunk": round(dt * 1e3, 3)}
    # the product check: the staged pieces and the one pass give the IEEE
    # sums on the host
    a0 = torch.empty(n, dtype=torch.float32).uniform_(-1, 1)
    h_dst.copy_(a0)
    staged(1)()
    torch.cuda.synchronize(dev)
    out["library_staged_verified"] = bool(torch.equal(h_dst, a0 + h_src))
    h_dst.copy_(a0)
    staged(n)()
    torch.cuda.synchronize(dev)
    out["library_one_pass_verified"] = bool(torch.equal(h_dst, a0 + h_src))
    # gloo_hip_reduce_staged with piece 0: zero-copy on these mapped buffers
    h_dst.copy_(a0)
    staged(0)()
    torch.cuda.synchronize(dev)
    out["library_default_verified"] = bool(torch.equal(h_dst, a0 + h_src))
    # the product check: the zero-copy kernel reads host memory correctly
    ref = d_dst.clone()
    d_src.copy_(h_src)
    want = ref + d_src
    hip.reduce_ptr("sum", "f32", ref.data_ptr(), hs, n, s.cuda_stream)
    torch.cuda.synchronize(dev)
    out["zero_copy_verified"] = bool(torch.equal(ref, want))
    out["gib_s_alg"] = out["serial"]["gib_s_alg"]
    out["ms_per_chunk"] = out["serial"]["ms_per_chunk"]
    out["note"] = "64 MiB fp32 chunk in pinned host memory; PCIe-bound, never the headline value"
    return out


CEILING_LIB = os.path.join(ROOT, "tools", "tune", "libceiling.so")
CEILING_PATTERN = 8  # hbm_ceiling.hip kP[8]: R2W1, unroll 2, 512 lanes (the product kernel's tile)


def stream_ceiling(torch, dev, stream, pairs, n, steps):
    """The chip's streaming rate for config 2's access mix, measured in the
    same run as the product kernel: the stripped kernel of
    tools/tune/hbm_ceiling.hip with reduce_vec_kernel's tile (raw nt buffer
    loads / stores, 16 B per lane, 512 lanes x 2 packets per stream, one tile
    per workgroup), two reads and one write IN PLACE (dst = dst + src over the
    same rotated 64 MiB pairs), timed exactly as the headline kernel (K
    back-to-back launches, fence-free events after launch 1 and launch K).
    No edge handling, no misalignment support, no dtype/op dispatch: what is
    left is the memory system's rate for 2R + 1W."""
    import ctypes
    if not os.path.exists(CEILING_LIB):
        return {"error": f"{CEILING_LIB} missing (built by __graft_entry__.build())"}
    L = ctypes.CDLL(CEILING_LIB)
    vp = ctypes.c_void_p
    L.ceil_run.argtypes = [ctypes.c_int, vp, vp, vp, vp, ctypes.c_size_t, vp]
    d4 = (ctypes.c_int * 4)()
    L.ceil_desc(CEILING_PATTERN, d4)
    if list(d4) != [2, 1, 2, 512] or (n * 4) % (512 * 2 * 16):
        return {"error": f"pattern {CEILING_PATTERN} is {list(d4)}; chunk not a whole number of tiles"}
    sink = torch.zeros(1024, dtype=torch.int32, device=dev)
    sh = stream.cuda_stream

    def launch(i):
        d, s = pairs[i % len(pairs)]
        rc = L.ceil_run(CEILING_PATTERN, d.data_ptr(), d.data_ptr(), s.data_ptr(), sink.data_ptr(), n * 4, sh)
        if rc:
            raise RuntimeError(f"ceil_run: {rc}")

    for i in range(3):
        launch(i)
    torch.cuda.synchronize(dev)
    e0, e1 = HipEvent(stream), HipEvent(stream)
    launch(0)
    e0.record()
    for i in range(1, steps):
        launch(i)
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_ms(e1) / (steps - 1)
    e0.destroy()
    e1.destroy()
    gbs = 3.0 * n * 4 / (ms / 1e3) / 1e9
    return {"kernel": "tools/tune/hbm_ceiling.hip stream_k<R=2, W=1, U=2, B=512> in place (stripped 2R+1W, same "
                      "tile, cache policy and rotation as the product kernel)",
            "kernel_avg_us": round(ms * 1e3, 3), "achieved_gbs": round(gbs, 1),
            "frac_of_peak": round(gbs / HBM_PEAK_GBS, 4)}


def xgmi_allreduce(torch, dist, hip, rank, world, dev, args, partial):
    """BASELINE config 3 (+ a config-4 sweep) at N > 1 ranks, one per GPU.

    Config 3: AllreduceRingChunked fp32 sum, 256 MiB per rank.  Chunks move
    GPU->GPU into the peer's HBM inbox (xGMI) and are reduced by the HIP
    kernel on the receiving GPU.  Default: the mesh plan (the ring's bytes,
    every link at once); variants: the mesh replayed as a hipGraph, the
    reference's (pipelined) ring route replayed and eager, the HOST workspace.  Reported: the slowest
    rank's time per allreduce, bus bandwidth, and the reduction kernels' own
    GiB/s measured with HIP events while the exchange runs (per-GPU
    efficiency vs the 1-GPU figure).
    Config 4: halving-doubling, 1 KiB .. 1 GiB per rank (x4 steps) for the
    derived mesh plan and the reference's exchange route, 4 sizes for the
    other variants.  Config 5: reduce-scatter of fp16 / bf16 buckets, all
    four ops.  New style: BCUBE allreduce and gloo::reduce, four sizes.
    `partial` collects each finished subsection, so a watchdog firing late
    still reports everything measured before it."""
    import tempfile
    # wall seconds per section on rank 0's clock (where an 8-GPU run spends its time)
    sections = {}
    partial["section_s"] = sections
    t_mark = [time.perf_counter()]

    def mark(name):
        now = time.perf_counter()
        sections[name] = round(now - t_mark[0], 1)
        t_mark[0] = now

    obj = [tempfile.mkdtemp(prefix="gloo_amd_bench_")] if rank == 0 else [None]
    dist.broadcast_object_list(obj, src=0)
    n = args.allreduce_mib * (1 << 20) // 4

    stores = [0]

    def store_url(name):
        """A store directory of its own for every context: a repeated
        variant must not read the keys an earlier context left behind."""
        stores[0] += 1
        return "file:%s/%s_%d" % (obj[0], name, stores[0])

    def gather(res):
        g = [None] * world
        dist.all_gather_object(g, res)
        return g

    def with_env(env, fn):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            return fn()
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

    # Result check of config 3 at every world size: rank r's input is
    # N(0,1) from seed (7, r); after run 1 the values at 4096 sampled
    # positions must equal the reference schedule's fold at those positions
    # (gloo/allreduce_ring_chunked.h:102-158: chunk pair q starts on rank q,
    # every later rank computes `local + incoming`), bit for bit; after the
    # last run every rank must hold the same bytes.
    import numpy as np
    sample = np.unique(np.random.default_rng(11).integers(0, n, 4096))
    x_np = np.random.default_rng([7, rank]).standard_normal(n, dtype=np.float32)
    x_all = gather(x_np[sample].tolist())
    chunks = 2 * world
    cs = max(256, (n + chunks - 1) // chunks)

    def expected_at_sample():
        xs = np.array(x_all, dtype=np.float32)  # [world][len(sample)]
        q = (sample // cs) // 2
        acc = xs[q, np.arange(len(sample))].copy()
        for j in range(1, world):
            acc = xs[(q + j) % world, np.arange(len(sample))] + acc
        return acc

    want_sample = expected_at_sample()

    def ring_once(launch="auto", workspace="device", mesh="1"):
        """launch: "auto" (the library's choice), "eager" (GLOO_AMD_GRAPH=0)
        or "graph" (GLOO_AMD_GRAPH=1)."""
        progress(f"config 3: ring_chunked launch={launch} workspace={workspace} mesh={mesh}")

        url = store_url("ring_%s_%s_%s" % (launch, workspace, mesh))  # taken first: every rank, same order

        def body():
            import hashlib
            buf = torch.from_numpy(x_np).to(dev)
            torch.cuda.synchronize(dev)
            ctx = hip.Context(rank, world, url,
                              device=dev.index, timeout_ms=60000)
            a = hip.Algorithm(ctx, "ring_chunked", "sum", "f32", [buf.data_ptr()], n, workspace=workspace)
            a.run()
            got = buf[torch.from_numpy(sample).to(dev)].cpu().numpy()
            ok_first = bool((got.view(np.uint32) == want_sample.view(np.uint32)).all())
            badmask = got.view(np.uint32) != want_sample.view(np.uint32)
            bad_first = int(badmask.sum())
            # first few mismatches: position, value, expected, this rank's input
            bad_detail = [[int(sample[i]), float(got[i]), float(want_sample[i]), float(x_np[sample[i]])]
                          for i in np.nonzero(badmask)[0][:3]]
            # timed: steady state (eager enqueue for these 32 MiB messages by default,
            # graph replay from run 3 on below 4 MiB messages, on the ring route, or with GLOO_AMD_GRAPH=1)
            times = []
            for _ in range(args.allreduce_iters):
                dist.barrier()
                t0 = time.perf_counter()
                a.run()
                times.append(time.perf_counter() - t0)
            graphed = a.mode()["graph"]
            # profiled: every chunk reduction bracketed by HIP events (eager)
            a.set_profiling(True)
            red_s = red_b = wait_s = 0.0
            for _ in range(3):
                dist.barrier()
                a.run()
                st = a.stats()
                red_s += st["reduce_s"]
                red_b += st["reduce_bytes"]
                wait_s += st["wait_s"]
            # steady state with device stamps: each reduce kernel records its
            # first-workgroup start / last-workgroup end on the GPU clock, so
            # the runs keep their launch mode, graph replay included (SURVEY
            # 8(e): the per-GPU reduce rate while the exchange runs)
            a.set_profiling(2)
            st_s = st_b = 0.0
            st_graph = []
            for it in range(2 + args.allreduce_iters):
                dist.barrier()
                a.run()
                st = a.stats()
                if it >= 2:  # run 1 re-enqueues, run 2 captures; replays after
                    st_s += st["reduce_s"]
                    st_b += st["reduce_bytes"]
                    st_graph.append(a.mode()["graph"])
            # fold + forward is off under event profiling and on (if the knob
            # allows) under stamps: mode() reports whether any run fused
            st_fused = a.mode()["fold_send"]
            a.set_profiling(0)
            torch.cuda.synchronize(dev)
            dig = hashlib.sha256(buf.cpu().numpy().view(np.uint8).tobytes()).hexdigest()
            a.close()
            ctx.close()
            return {"ms": [round(t * 1e3, 3) for t in times], "reduce_s": red_s, "reduce_b": red_b,
                    "wait_ms_per_run": round(wait_s / 3 * 1e3, 3), "first_run_ok": ok_first,
                    "first_run_bad_samples": bad_first, "first_run_bad_detail": bad_detail, "digest": dig,
                    "graph": graphed, "stamp_s": st_s, "stamp_b": st_b, "stamp_graph": all(st_graph),
                    "stamp_fused": bool(st_fused)}
        try:
            env = {"GLOO_AMD_MESH": mesh}
            if launch != "auto":
                env["GLOO_AMD_GRAPH"] = "0" if launch == "eager" else "1"
            res = with_env(env, body)
        except Exception as e:  # noqa: BLE001
            res = {"error": repr(e)}
        gathered = gather(res)
        errs = [g["error"] for g in gathered if "error" in g]
        if errs:
            return {"launch": launch, "error": errs[0],
                    "errors_per_rank": [g.get("error") for g in gathered]}
        ms = sorted(max(g["ms"][i] for g in gathered) for i in range(args.allreduce_iters))
        t = ms[len(ms) // 2] / 1e3
        per_gpu = [g["reduce_b"] / g["reduce_s"] / GIB for g in gathered if g["reduce_s"] > 0]
        fused = all(g["stamp_fused"] for g in gathered)
        busbw = 2 * (world - 1) / world * n * 4 / t
        links = link_bounds(world, n * 4, t, link["figures"])
        return {"plan": "mesh" if mesh == "1" and world <= 8 else "ring", "launch": launch,
                "workspace": workspace, "graph": all(g["graph"] for g in gathered),
                "ms_p50": round(t * 1e3, 3), "algbw_gib_s": round(n * 4 / t / GIB, 2),
                "busbw_gib_s": round(busbw / GIB, 2), **links,
                "schedule": ("%s%s" % ("mesh" if mesh == "1" and world <= 8 else "ring",
                                       ", fold + forward fused" if fused else ", unfused (fold, then sends)")),
                "reduce_kernel_gib_s_per_gpu_eager_events": [round(x, 1) for x in per_gpu],
                "reduce_kernel_gib_s_per_gpu": [round(g["stamp_b"] / g["stamp_s"] / GIB, 1) if g["stamp_s"] > 0
                                                else None for g in gathered],
                "reduce_kernel_timing": ("device stamps inside the reduce kernels (first workgroup start to last "
                                         "workgroup end%s), %d %s runs per rank" %
                                         (", forward stores included: the fused fold + forward launch as it ships"
                                          if fused else "",
                                          args.allreduce_iters, "graph-replayed" if all(g["stamp_graph"] for g in gathered)
                                          else "eagerly enqueued (the mesh default from 4 MiB messages)")),
                "host_wait_ms_per_run_max_profiled": max(g["wait_ms_per_run"] for g in gathered),
                "verified": bool(all(g["first_run_ok"] for g in gathered) and
                                 len({g["digest"] for g in gathered}) == 1),
                "first_run_bad_samples_per_rank": [g["first_run_bad_samples"] for g in gathered],
                "first_run_bad_detail_per_rank": [g["first_run_bad_detail"] for g in gathered],
                "final_digests_equal": len({g["digest"] for g in gathered}) == 1,
                "verify": "run 1 vs the reference ring fold at 4096 sampled positions on every rank, "
                          "bit-exact; after the last run every rank's 256 MiB digest equal"}

    ngpu = torch.cuda.device_count()
    # the link figures the ring / mesh bounds use (link_figures): measured by
    # rank 0 over its direct xGMI links, null with the reason on one GPU
    link = link_figures(torch, dist, rank, world, n * 4)
    partial["link"] = link
    # default: the mesh plan (batched sends = one multi-destination copy kernel)
    ring = ring_once()
    partial["config"] = "allreduce_ring_chunked fp32 sum, %d ranks, %d MiB/rank" % (world, args.allreduce_mib)
    partial["data_path"] = "xGMI peer copies" if ngpu >= world else f"{world} ranks on {ngpu} GPU(s)"
    partial.update(ring)
    if "error" in ring:
        return dict(partial)
    variants = {}
    partial["variants"] = variants
    # the launch modes and routes that ship (the knobs that switched copy
    # engines, store flavours and completion protocols are gone: each lost
    # its A/B, DESIGN.md §4 / INTEGRATION.md §4)
    specs = {"ring_graph": ("auto", "device", "0"), "ring_eager": ("eager", "device", "0"),
             "mesh_graph": ("graph", "device", "1"), "mesh_host_workspace": ("auto", "host", "1")}
    chosen = (args.config3_variants.split(",") if args.config3_variants
              else ["ring_graph"] if args.quick else list(specs))
    for k, name in enumerate(chosen):
        launch, workspace, mesh = specs[name]
        variants[name if name not in variants else "%s#%d" % (name, k + 1)] = ring_once(launch, workspace, mesh)
    partial["ipc_pool"] = hip.ipc_stats()
    mark("config3")
    if args.config3_only:
        return dict(partial)

    def runner_samples(run_once):
        """gloo/benchmark/runner.cc:311-363: 5 warm-up runs; an iteration
        count from the median warm-up time (the slowest rank's, so every rank
        agrees), runs timed back to back, the count grown x2 until a batch
        lasts args.sweep_seconds (the reference's default 2 s; less here so
        the driver's run stays bounded) or reaches 10,000.  Returns this
        rank's per-run seconds of the last batch."""
        warm = []
        for _ in range(5):
            t0 = time.perf_counter()
            run_once()
            warm.append(time.perf_counter() - t0)
        med = torch.tensor([sorted(warm)[2]], dtype=torch.float64)
        dist.all_reduce(med, op=dist.ReduceOp.MAX)
        iters_ = max(1, int(args.sweep_seconds / max(float(med[0]), 1e-9)))
        while True:
            iters_ = min(iters_, 10000)
            dist.barrier()
            ts = []
            for _ in range(iters_):
                t0 = time.perf_counter()
                run_once()
                ts.append(time.perf_counter() - t0)
            tot = torch.tensor([sum(ts)], dtype=torch.float64)
            dist.all_reduce(tot, op=dist.ReduceOp.MIN)
            if float(tot[0]) >= args.sweep_seconds or iters_ >= 10000:
                return ts
            iters_ *= 2

    short_sizes = (1 << 10, 64 << 10, 1 << 20, 64 << 20)
    full_sizes = tuple(1 << lg for lg in range(10, 31, 2))  # config 4: 1 KiB .. 1 GiB per rank
    iters = 20

    def hd_sweep(label, env, sizes=short_sizes):
        def body():
            hd = []
            for nbytes in sizes:
                progress(f"halving_doubling {label} {nbytes} B")
                m = max(1, nbytes // 4)
                url = store_url("hd_%s_%d" % (label, nbytes))
                try:
                    # rank r contributes r + 1: run 1 must give P(P+1)/2 in
                    # every element (exact in fp32), whatever the fold order
                    b2 = torch.full((m,), float(rank + 1), device=dev)
                    torch.cuda.synchronize(dev)
                    ctx2 = hip.Context(rank, world, url,
                                       device=dev.index, timeout_ms=60000)
                    a2 = hip.Algorithm(ctx2, "halving_doubling", "sum", "f32", [b2.data_ptr()], m)
                    a2.run()
                    ok = bool((b2 == world * (world + 1) / 2).all())
                    b2.fill_(1.0)
                    ts = runner_samples(a2.run)
                    md = a2.mode()
                    a2.close()
                    ctx2.close()
                    hd.append({"bytes": nbytes, "us": [round(t * 1e6, 1) for t in ts], "graph": md["graph"],
                               "interp": md["interp"], "ok": ok})
                except Exception as e:  # noqa: BLE001
                    hd.append({"bytes": nbytes, "error": repr(e)})
            return hd
        hd_all = gather(with_env(env, body))
        summary = []
        for i, nbytes in enumerate(sizes):
            if any("error" in h[i] for h in hd_all):
                summary.append({"bytes": nbytes,
                                "error": next(h[i]["error"] for h in hd_all if "error" in h[i])})
                continue
            k_all = min(len(h[i]["us"]) for h in hd_all)
            per = sorted(max(h[i]["us"][k] for h in hd_all) for k in range(k_all))
            p50, p99 = per[len(per) // 2], per[min(len(per) - 1, int(len(per) * 0.99))]
            summary.append({"bytes": nbytes, "us_p50": p50, "us_p99": p99, "us_max": per[-1],
                            "samples": len(per),
                            "verified": all(h[i]["ok"] for h in hd_all),
                            "launch": "interp" if all(h[i]["interp"] for h in hd_all)
                            else "graph" if all(h[i]["graph"] for h in hd_all) else "eager",
                            "busbw_gib_s": round(2 * (world - 1) / world * nbytes / (p50 / 1e6) / GIB, 3)})
        return summary

    # mesh = the derived mesh plan (default); reference_route = the
    # reference's halving/doubling exchange (GLOO_AMD_MESH=0)
    hd_variants = {"mesh": {},
                   "mesh_eager": {"GLOO_AMD_GRAPH": "0", "GLOO_AMD_INTERP": "0"},
                   "mesh_no_interp": {"GLOO_AMD_INTERP": "0"},
                   "reference_route": {"GLOO_AMD_MESH": "0"},
                   "reference_route_eager": {"GLOO_AMD_MESH": "0", "GLOO_AMD_GRAPH": "0", "GLOO_AMD_INTERP": "0"}}
    # With a GPU per rank, a larger sliced-interpreter cap (DESIGN.md §8
    # "Remaining" 4): 8 MiB messages (64 MiB per rank at P = 8) run sliced
    # instead of eager.  Only there: ranks sharing a GPU cannot all keep 128
    # workgroups resident, and their device-side waits time out.
    one_rank_per_gpu = world <= torch.cuda.device_count()
    if one_rank_per_gpu and world > 1:
        hd_variants["mesh_slices_128"] = {"GLOO_AMD_INTERP_MAX_SLICES": "128"}
    hd_summary = {}
    partial["halving_doubling"] = hd_summary
    for k, v in hd_variants.items():
        if args.quick and k not in ("mesh", "reference_route"):
            continue
        big = k in ("mesh", "reference_route") and not args.quick
        sizes = (16 << 20, 64 << 20) if k == "mesh_slices_128" else full_sizes if big else short_sizes
        hd_summary[k] = hd_sweep(k, v, sizes)
    mark("config4_halving_doubling")

    # Config 5: reduce-scatter (HD), fp16 / bf16 buckets, every op, 16 Mi
    # elements per rank, recvElems = an even split.
    def rs_once(dtype, op, env, m=16 << 20):
        progress(f"reduce_scatter {dtype} {op} {env} {m}")
        url = store_url("rs_%s_%s_%s_%d" % (dtype, op, env.get("GLOO_AMD_MESH", "1"), m))

        def body():
            recv = [m // world + (1 if r < m % world else 0) for r in range(world)]
            # rank r contributes 1 + r % 2: every op's result is exact in
            # fp16 / bf16 for P <= 8, so run 1's block is checked whole
            vals = [1.0 + r % 2 for r in range(world)]
            want = {"sum": sum(vals), "product": float(np.prod(vals)), "max": max(vals), "min": min(vals)}[op]
            b = torch.full((m,), vals[rank], dtype=torch.float16 if dtype == "f16" else torch.bfloat16, device=dev)
            torch.cuda.synchronize(dev)
            c = hip.Context(rank, world, url, device=dev.index, timeout_ms=60000)
            a = hip.Algorithm(c, "reduce_scatter", op, dtype, [b.data_ptr()], m, recv_elems=recv)
            a.run()
            ok = bool((b[:recv[rank]].float() == want).all())
            a.run()
            ts = []
            for _ in range(10):
                dist.barrier()
                t0 = time.perf_counter()
                a.run()
                ts.append(time.perf_counter() - t0)
            a.close()
            c.close()
            return {"us": [round(t * 1e6, 1) for t in ts], "ok": ok}
        try:
            res = with_env(env, body)
        except Exception as e:  # noqa: BLE001
            res = {"error": repr(e)}
        g = gather(res)
        if any("error" in x for x in g):
            return {"dtype": dtype, "op": op, "error": next(x["error"] for x in g if "error" in x)}
        per = sorted(max(x["us"][k] for x in g) for k in range(10))
        nbytes = m * 2
        return {"dtype": dtype, "op": op, "route": "reference" if env.get("GLOO_AMD_MESH") == "0" else "mesh",
                "elements_per_rank": m, "us_p50": per[5], "us_max": per[-1],
                "verified": all(x["ok"] for x in g),
                "busbw_gib_s": round((world - 1) / world * nbytes / (per[5] / 1e6) / GIB, 2)}

    rs_summary = [rs_once(dt, op, {}) for dt in ("f16", "bf16") for op in ("sum", "product", "min", "max")]
    if args.quick:
        partial["reduce_scatter"] = rs_summary
        mark("config5_reduce_scatter")
        return dict(partial)
    rs_summary += [rs_once(dt, "sum", {"GLOO_AMD_MESH": "0"}) for dt in ("f16", "bf16")]
    partial["reduce_scatter"] = rs_summary
    # the other two bucket sizes of SURVEY 8(d) config 5: 1 Mi and 64 Mi elements per rank
    for m in (1 << 20, 64 << 20):
        rs_summary += [rs_once(dt, "sum", env, m) for dt in ("f16", "bf16") for env in ({}, {"GLOO_AMD_MESH": "0"})]

    # New-style function API: gloo::allreduce RING / BCUBE
    # and gloo::reduce to rank 0, fp32 sum, separate input and output; the
    # derived mesh route (default) and the reference's exchange route.
    def newstyle(kind, nbytes, env=None):
        progress(f"new style {kind} {nbytes} B {env}")
        url = store_url("ns_%s_%d_%s" % (kind, nbytes, bool(env)))

        def body():
            m = max(1, nbytes // 4)
            inp = torch.ones(m, device=dev)
            outp = torch.zeros(m, device=dev)
            torch.cuda.synchronize(dev)
            c = hip.Context(rank, world, url,
                            device=dev.index, timeout_ms=60000)

            def call():
                if kind in ("ring", "bcube"):
                    hip.allreduce(c, [outp.data_ptr()], m, "f32", "sum", inputs=[inp.data_ptr()], algorithm=kind)
                else:
                    hip.reduce_to_root(c, outp.data_ptr(), m, "f32", 0, "sum", input=inp.data_ptr())
            call()
            call()
            ts = []
            for _ in range(10):
                dist.barrier()
                t0 = time.perf_counter()
                call()
                ts.append(time.perf_counter() - t0)
            ok = bool((outp[:: max(1, m // 1024)] == world).all()) if (kind != "reduce" or rank == 0) else True
            c.close()
            return {"us": [round(t * 1e6, 1) for t in ts], "ok": ok}
        try:
            res = with_env(env or {}, body)
        except Exception as e:  # noqa: BLE001
            res = {"error": repr(e)}
        g = gather(res)
        if any("error" in x for x in g):
            return {"bytes": nbytes, "error": next(x["error"] for x in g if "error" in x)}
        per = sorted(max(x["us"][k] for x in g) for k in range(10))
        return {"bytes": nbytes, "us_p50": per[5], "us_max": per[-1], "verified": all(x["ok"] for x in g)}

    ns_sizes = (64 << 10, 1 << 20, 16 << 20, 256 << 20)
    ns = {}
    partial["new_style"] = ns
    mark("config5_reduce_scatter")
    ref_route = {"GLOO_AMD_MESH": "0"}
    for kind, label in (("ring", "ring_allreduce"), ("bcube", "bcube_allreduce"), ("reduce", "reduce_to_root0")):
        ns[label] = [newstyle(kind, b) for b in ns_sizes]
        ns[label + "_reference_route"] = [newstyle(kind, b, ref_route) for b in ns_sizes[2:]]
    mark("new_style")
    dist.barrier()
    if rank == 0:
        import shutil
        shutil.rmtree(obj[0], ignore_errors=True)
    return dict(partial)


# The link figures the xGMI bounds are set from: the
# product's own copy kernel (64 and 256 workgroups per copy) and the runtime's
# peer copy, one peer one direction, one peer both directions at once, and
# all P-1 peers at once from one GPU (the mesh send pattern, one
# multi-destination launch) — SURVEY 8(e); gloo/benchmark/runner.cc:497-506.
LINK_FIGURES = ("kernel64_one_peer_one_dir", "kernel256_one_peer_one_dir", "memcpy_one_peer_one_dir",
                "kernel64_one_peer_both_dirs", "memcpy_one_peer_both_dirs",
                "kernel64_all_peers_one_gpu", "memcpy_all_peers_one_gpu")
# which figure bounds which route: a ring hop is one link in one direction
# (the copy kernel: the product's eager SEND engine); a mesh phase sends to
# every peer at once (one multi-destination copy kernel launch)
RING_BOUND_FIGURE = "kernel64_one_peer_one_dir"
MESH_BOUND_FIGURE = "kernel64_all_peers_one_gpu"


def link_bounds(world, nbytes, t, figures):
    """The link-bound fields of a config-3 line: ring and mesh lower bounds
    on the allreduce time of `nbytes` per rank over `world` ranks, from the
    named figures (GB/s per link), and the measured time `t` (s) against
    them.  A missing figure gives null bounds with the reason.
      ring: 2(P-1) hops of S/P, each over one link: 2(P-1)/P * S / B_ring
      mesh: two phases, each moving S/P over every link at once: 2 S/P / B_mesh
      busbw = 2(P-1)/P * S / t (the nccl-tests bus bandwidth)"""
    busbw = 2 * (world - 1) / world * nbytes / t
    out = {}
    for route, name, traffic in (("ring", RING_BOUND_FIGURE, 2 * (world - 1) / world * nbytes),
                                 ("mesh", MESH_BOUND_FIGURE, 2 * nbytes / world)):
        f = figures.get(name) or {}
        B = f.get("GBps_per_link") or f.get("GBps")
        out[route + "_bound_figure"] = name
        if B:
            out[route + "_link_bound_ms"] = round(traffic / (B * 1e9) * 1e3, 3)
            out["frac_of_%s_link_bound" % route] = round(traffic / (B * 1e9) / t, 4)
        else:
            out[route + "_link_bound_ms"] = None
            out["frac_of_%s_link_bound" % route] = None
            out[route + "_bound_why"] = f.get("why", "figure not measured")
    ring = figures.get(RING_BOUND_FIGURE) or {}
    out["busbw_frac_of_link"] = round(busbw / (ring["GBps"] * 1e9), 4) if ring.get("GBps") else None
    return out


def link_figures(torch, dist, rank, world, nbytes):
    """LINK_FIGURES measured by rank 0 alone on the GPUs it sees (every rank
    joins the barriers), best of 5 timed with HIP events; each figure is
    {"GBps"...} or {"GBps": None, "why": ...}."""
    ngpu = torch.cuda.device_count()
    res = [None]
    dist.barrier()
    if rank == 0:
        figs = {}
        if ngpu < 2:
            why = f"{world} ranks on {ngpu} GPU(s): no xGMI link to measure"
            figs = {k: {"GBps": None, "why": why} for k in LINK_FIGURES}
        else:
            try:
                figs = _measure_links(torch, min(ngpu, max(2, world)), nbytes)
            except Exception as e:  # noqa: BLE001
                figs = {k: {"GBps": None, "why": repr(e)} for k in LINK_FIGURES}
        res[0] = {"unit": "GB/s (1e9 B/s)", "bytes": nbytes, "figures": figs,
                  "ring_bound_figure": RING_BOUND_FIGURE, "mesh_bound_figure": MESH_BOUND_FIGURE}
    dist.broadcast_object_list(res, src=0)
    return res[0]


def _measure_links(torch, P, nbytes):
    import gloo_amd as hip
    rt = ctypes.CDLL("libamdhip64.so.7")
    for a in range(P):  # peer access both ways between GPU 0 and every peer
        for b in ((range(1, P)) if a == 0 else (0,)):
            rt.hipSetDevice(a)
            rt.hipDeviceEnablePeerAccess(b, 0)
    rt.hipGetLastError()
    rt.hipSetDevice(0)
    dev = [torch.device("cuda", g) for g in range(P)]
    src0 = torch.empty(nbytes, dtype=torch.uint8, device=dev[0])
    dst = [None] + [torch.empty(nbytes, dtype=torch.uint8, device=dev[g]) for g in range(1, P)]
    src1 = torch.empty(nbytes, dtype=torch.uint8, device=dev[1])
    dst0 = torch.empty(nbytes, dtype=torch.uint8, device=dev[0])
    s0 = torch.cuda.Stream(dev[0])
    s1 = torch.cuda.Stream(dev[1])
    peers = [torch.cuda.Stream(dev[0]) for _ in range(1, P)]

    def timed(stream, fn, reps=6):
        best = None
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        return best / 1e3

    figs = {}
    for blocks in (64, 256):
        t = timed(s0, lambda: hip.copy_kernel(dst[1].data_ptr(), src0.data_ptr(), nbytes, blocks, s0.cuda_stream))
        figs[f"kernel{blocks}_one_peer_one_dir"] = {"GBps": round(nbytes / t / 1e9, 2)}

    def memcpy_one():
        with torch.cuda.stream(s0):
            dst[1].copy_(src0, non_blocking=True)
    figs["memcpy_one_peer_one_dir"] = {"GBps": round(nbytes / timed(s0, memcpy_one) / 1e9, 2)}

    def both(kernel):
        # GPU 0 -> 1 on GPU 0's stream, GPU 1 -> 0 on GPU 1's, started together
        best = None
        for _ in range(6):
            torch.cuda.synchronize(dev[0])
            torch.cuda.synchronize(dev[1])
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(2)]
            evs[0][0].record(s0)
            evs[1][0].record(s1)
            if kernel:
                hip.copy_kernel(dst[1].data_ptr(), src0.data_ptr(), nbytes, 64, s0.cuda_stream)
                hip.copy_kernel(dst0.data_ptr(), src1.data_ptr(), nbytes, 64, s1.cuda_stream)
            else:
                with torch.cuda.stream(s0):
                    dst[1].copy_(src0, non_blocking=True)
                with torch.cuda.stream(s1):
                    dst0.copy_(src1, non_blocking=True)
            evs[0][1].record(s0)
            evs[1][1].record(s1)
            evs[0][1].synchronize()
            evs[1][1].synchronize()
            ms = max(evs[0][0].elapsed_time(evs[0][1]), evs[1][0].elapsed_time(evs[1][1]))
            best = ms if best is None else min(best, ms)
        t = best / 1e3
        return {"GBps": round(nbytes / t / 1e9, 2), "GBps_total": round(2 * nbytes / t / 1e9, 2),
                "how": "per direction, both directions at once (the slower one's time)"}
    figs["kernel64_one_peer_both_dirs"] = both(True)
    figs["memcpy_one_peer_both_dirs"] = both(False)

    k = P - 1
    t = timed(s0, lambda: hip.copy_kernel_multi([d.data_ptr() for d in dst[1:]], [src0.data_ptr()] * k, nbytes, 64,
                                                s0.cuda_stream))
    figs["kernel64_all_peers_one_gpu"] = {"peers": k, "GBps_per_link": round(nbytes / t / 1e9, 2),
                                          "GBps_total": round(k * nbytes / t / 1e9, 2),
                                          "how": "one multi-destination copy launch, 64 workgroups per peer"}

    def memcpy_all():
        fork = torch.cuda.Event()
        fork.record(s0)
        joins = []
        for j, st in enumerate(peers):
            st.wait_event(fork)
            with torch.cuda.stream(st):
                dst[j + 1].copy_(src0, non_blocking=True)
            e = torch.cuda.Event()
            e.record(st)
            joins.append(e)
        for e in joins:
            s0.wait_event(e)
    t = timed(s0, memcpy_all)
    figs["memcpy_all_peers_one_gpu"] = {"peers": k, "GBps_per_link": round(nbytes / t / 1e9, 2),
                                        "GBps_total": round(k * nbytes / t / 1e9, 2),
                                        "how": "one peer copy per stream, forked and joined on GPU 0"}
    del src0, dst, src1, dst0
    torch.cuda.empty_cache()
    return figs


class HipEvent:
    """A timing event of the HIP runtime torch has loaded (same soname),
    created with hipEventDisableSystemFence (hip_runtime_api.h): recorded
    between two kernels it stalls the stream ~1 us instead of the ~2.9 us of
    a default event's system-scope release (profiles/round2/r2zv_*)."""
    kDisableSystemFence = 0x20000000
    _rt = None

    def __init__(self, stream):
        if HipEvent._rt is None:
            HipEvent._rt = ctypes.CDLL("libamdhip64.so.7")
        self.stream = ctypes.c_void_p(stream.cuda_stream)
        self.h = ctypes.c_void_p()
        rc = HipEvent._rt.hipEventCreateWithFlags(ctypes.byref(self.h), ctypes.c_uint(self.kDisableSystemFence))
        if rc != 0:
            raise RuntimeError(f"hipEventCreateWithFlags failed: {rc}")

    def record(self):
        rc = HipEvent._rt.hipEventRecord(self.h, self.stream)
        if rc != 0:
            raise RuntimeError(f"hipEventRecord failed: {rc}")

    def spin(self):
        """Busy-poll until the stream has passed this event (hipEventQuery;
        hipErrorNotReady = 600), so the host sees the end of the timed work
        without a blocking wait's wake-up latency."""
        while True:
            rc = HipEvent._rt.hipEventQuery(self.h)
            if rc != 600:
                if rc != 0:
                    raise RuntimeError(f"hipEventQuery failed: {rc}")
                return

    def elapsed_ms(self, other):
        ms = ctypes.c_float()
        rc = HipEvent._rt.hipEventElapsedTime(ctypes.byref(ms), self.h, other.h)
        if rc != 0:
            raise RuntimeError(f"hipEventElapsedTime failed: {rc}")
        return ms.value

    def destroy(self):
        """Explicitly, while the runtime is up (never from __del__ at exit)."""
        if self.h:
            HipEvent._rt.hipEventDestroy(self.h)
            self.h = ctypes.c_void_p()


def watchdog_line(out, partial, reason, efficiency, tries=5):
    """The JSON line a firing watchdog prints.  It runs on the watchdog thread
    while the main thread may still be filling `partial`, so a snapshot can
    race ("dictionary changed size during iteration"): retry it, and fall back
    to the line without the partial results if it keeps failing."""
    note = "the N>1 section timed out: the job exits 3 after this line"
    for _ in range(tries):
        try:
            snap = json.loads(json.dumps(partial))
            line = dict(out, xgmi_allreduce=dict(snap, error="watchdog: " + reason),
                        per_gpu_efficiency=efficiency(snap), value_note=note)
            return json.dumps(line)
        except Exception:  # noqa: BLE001
            time.sleep(0.05)
    line = {k: v for k, v in dict(out).items() if k != "per_gpu_efficiency"}
    line.update(xgmi_allreduce={"error": "watchdog: " + reason + " (partial results unreadable)"}, value_note=note)
    return json.dumps(line)


class Watchdog:
    """Fires on_fire(reason) once the section has gone `idle_s` without a
    progress() line (every rank's sections end in a gather, so one hung rank
    stalls them all) or `total_s` in all; cancel() stops it."""

    def __init__(self, idle_s, total_s, on_fire):
        import threading
        self.stop = threading.Event()
        t0 = time.time()
        _LAST_PROGRESS[0] = t0

        def loop():
            while not self.stop.wait(min(1.0, idle_s / 4)):
                now = time.time()
                if now - _LAST_PROGRESS[0] > idle_s:
                    return on_fire("no progress for %.0f s" % (now - _LAST_PROGRESS[0]))
                if now - t0 > total_s:
                    return on_fire("section exceeded %.0f s" % total_s)
        self.t = threading.Thread(target=loop, daemon=True)
        self.t.start()

    def cancel(self):
        self.stop.set()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world == 1:
        sys.exit(relaunch_distributed(args))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist
    import gloo_amd as hip

    if world > 1:
        # (PyTorch's bundled Gloo prints its "[Gloo] Rank … connected" lines
        # with std::cout too: stdout carries only the JSON line)
        with stdout_fd_to_stderr():
            dist.init_process_group("gloo", rank=rank, world_size=world)
    # one GPU per rank; ranks wrap around the visible GPUs (rehearsals of the
    # multi-rank path on a 1-GPU box put every rank on cuda:0)
    dev = torch.device(f"cuda:{local_rank % max(1, torch.cuda.device_count())}")
    torch.cuda.set_device(dev)
    hip.set_variant(args.variant)

    n = args.chunk_mib * (1 << 20) // 4
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    pairs = [(torch.rand(n, device=dev, generator=g) * 2 - 1,
              torch.rand(n, device=dev, generator=g) * 2 - 1) for _ in range(args.pairs)]
    # 1 % of the lanes hold +-0, denormals and +-inf
    specials = torch.tensor([0.0, -0.0, 1e-40, -1e-40, float("inf"), float("-inf")], device=dev)
    for d, s in pairs:
        for t, off in ((d, 0), (s, 50)):
            idx = torch.arange(off, n, 100, device=dev)
            t[idx] = specials[torch.arange(idx.numel(), device=dev) % specials.numel()]
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    def step(i):
        d, s = pairs[i % len(pairs)]
        hip.reduce_ptr("sum", "f32", d.data_ptr(), s.data_ptr(), n, sh)

    progress(f"config 2: {args.warmup} warmup + {args.steps} timed steps")
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize(dev)

    # Timed region: barrier + sync on both sides, exactly K back-to-back
    # launches.  Kernel duration: two HIP events on the launch stream, the
    # first recorded right AFTER launch 1 is enqueued and the second after
    # launch K, so region / (K - 1) is the launch-to-launch time of kernels
    # 2..K running back to back, dispatch boundaries included.  (An event
    # recorded before launch 1 reaches the idle GPU first and would add launch
    # 1's host submission latency.)  The events are created with
    # hipEventDisableSystemFence: a default event between two kernels is a
    # marker with a system-scope release that stalls the stream ~2.9 us; this
    # one ~1.0 us (profiles/round2/r2zv_event_bubble.jsonl), so the region
    # holds 1 us of marker instead of 3.
    e_start = HipEvent(stream)
    e_end = HipEvent(stream)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    skip = 1 if args.steps >= 2 else 0   # K = 1: the whole single launch
    for i in range(skip):
        step(i)
    e_start.record()
    for i in range(skip, args.steps):
        step(i)
    e_end.record()
    e_end.spin()                 # the end of the K launches, seen without a blocking wait's wake-up
    torch.cuda.synchronize(dev)  # (returns at once: nothing else is queued)
    # each rank's own K steps; the slowest rank's time is taken below (MAX
    # over ranks), so the closing barrier's own latency stays outside
    wall = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    region_ms = e_start.elapsed_ms(e_end)
    kern_ms = region_ms / (args.steps - skip)
    e_start.destroy()
    e_end.destroy()

    t_local = torch.tensor([wall], dtype=torch.float64)
    k_all = torch.tensor([kern_ms], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t_local, op=dist.ReduceOp.MAX)
        k_list = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(k_list, k_all)
        per_rank_kernel_ms = [float(x) for x in k_list]
    else:
        per_rank_kernel_ms = [kern_ms]
    tmax = float(t_local[0])

    # the access mix's streaming ceiling, same run, same buffers, after the
    # timed region (in the driver-run line)
    ceiling = None
    if world == 1 and args.steps >= 2:
        try:
            ceiling = stream_ceiling(torch, dev, stream, pairs, n, args.steps)
        except (OSError, RuntimeError) as e:  # pragma: no cover
            ceiling = {"error": repr(e)}

    alg_bytes = 3.0 * n * 4                       # 2 reads + 1 write per element
    value = world * args.steps * alg_bytes / tmax / GIB
    achieved_gbs = alg_bytes / (kern_ms / 1e3) / 1e9

    out = None
    if rank == 0:
        traffic = None
        if os.path.exists(args.traffic_json):
            try:
                tj = json.load(open(args.traffic_json))
                if tj.get("elements") == n:
                    traffic = tj.get("hbm_bytes_per_launch")
            except (OSError, ValueError):
                traffic = None
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(tmax * 1e3 / args.steps, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": WORKLOAD, "chunk_bytes": n * 4, "elements": n,
                       "op": "sum", "form": "in-place dst += src (ReductionFunction::call)",
                       "rotated_pairs": args.pairs, "footprint_mib": 2 * args.pairs * args.chunk_mib,
                       "inputs": "U(-1,1), 1 % of lanes +-0 / denormal / +-inf",
                       "parallelism": f"{world} independent GPU(s), no data-path collective",
                       "kernel_variant": args.variant},
            "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "algorithmic_bytes_per_launch": int(alg_bytes),
                         "kernel_avg_us": round(kern_ms * 1e3, 3),
                         "per_rank_kernel_avg_us": [round(x * 1e3, 3) for x in per_rank_kernel_ms],
                         "event_region_ms": round(region_ms, 4),
                         "event_region_launches": args.steps - skip,
                         "timing": ("HIP events (hipEventDisableSystemFence) after launch 1 and after launch K "
                                    "on the launch stream, / (K - 1)")},
            "per_gpu_gib_s": round(value / world, 2),
            "kernel_gib_s": round(alg_bytes / (kern_ms / 1e3) / GIB, 2),
        }
        if world == 1:
            if ceiling and "achieved_gbs" in ceiling:
                out["roofline"]["ceiling_gbs"] = ceiling["achieved_gbs"]
                out["roofline"]["frac_of_ceiling"] = round(achieved_gbs / ceiling["achieved_gbs"], 4)
            out["roofline"]["ceiling"] = ceiling
            if not args.no_host_staged:
                out["host_staged"] = host_staged(torch, hip, n, dev)
            if not args.no_cpu:
                out["cpu_baseline"] = cpu_baseline(args, n)

    if world > 1 and not args.no_allreduce:
        # A failure in the collective must never cost the headline line: every
        # rank arms a watchdog; if it fires, rank 0 prints the headline with
        # the section marked as timed out, and the process exits.
        partial = {}

        def efficiency_of(xr, data_path):
            """each GPU's reduce-kernel GiB/s while the config-3
            exchange runs (device stamps, steady-state runs) over the same GPU's
            config-2 kernel GiB/s measured above in this run."""
            per = xr.get("reduce_kernel_gib_s_per_gpu") or []
            one = [alg_bytes / (k / 1e3) / GIB for k in per_rank_kernel_ms]
            eff = [p / o for p, o in zip(per, one) if p]
            if len(eff) != world:
                return {"value": None, "why": xr.get("error", "no stamped reduce timing from every rank"),
                        "data_path": data_path}
            return {"value": round(min(eff), 4), "mean": round(sum(eff) / len(eff), 4),
                    "per_rank": [round(e, 4) for e in eff],
                    "reduce_gib_s_during_allreduce": [round(p, 1) for p in per],
                    "one_gpu_kernel_gib_s": [round(o, 1) for o in one],
                    "schedule": xr.get("schedule"),
                    "how": ("min over ranks of (config-3 mesh allreduce reduce-kernel GiB/s, device stamps over "
                            "steady-state runs, bytes = the fold's (P + 1) reads and writes) / (the same GPU's "
                            "config-2 64 MiB kernel GiB/s in this run)"),
                    "data_path": data_path}

        def efficiency(xr):
            """Twice: SURVEY 8(e)'s definition on the unfused mesh (a pure
            fold kernel), and the default schedule as it ships (fold and
            forward in one launch, its forward stores inside the stamps)."""
            base = xr.get("data_path") or partial.get("data_path")
            # the unfused fold: the default run's event-profiled runs (events
            # need a pure fold kernel between them, so those runs are unfused)
            unf = {"reduce_kernel_gib_s_per_gpu": xr.get("reduce_kernel_gib_s_per_gpu_eager_events"),
                   "error": xr.get("error")}
            res = efficiency_of(unf, f"{base}; unfused mesh (event-profiled runs): fold kernel, then the sends")
            fused = efficiency_of(xr, f"{base}; default schedule: {xr.get('schedule', 'mesh')}")
            if fused.get("value") and "fused" in (xr.get("schedule") or "") and "unfused" not in xr["schedule"]:
                # the fused launch also stores each owner's range to its P - 1
                # peers: (P + 1) fold streams + (P - 1) forward streams
                k = 2 * world / (world + 1)
                fused["value_incl_forward_bytes"] = round(fused["value"] * k, 4)
                fused["forward_note"] = ("value counts the fold's (P + 1) streams only; value_incl_forward_bytes "
                                         "adds the (P - 1) forward stores the same launch makes (x 2P / (P + 1))")
            res["fused_default"] = fused
            return res

        def fire(reason):
            try:
                if rank == 0:
                    print(watchdog_line(out, partial, reason, efficiency), flush=True)
            finally:
                # a hung section must show in the driver's record: non-zero exit
                os._exit(3)

        progress("N>1 sections")
        wd = Watchdog(args.watchdog_seconds, args.watchdog_total_seconds, fire)
        xr = xgmi_allreduce(torch, dist, hip, rank, world, dev, args, partial)
        wd.cancel()
        if rank == 0:
            out["xgmi_allreduce"] = xr
            out["per_gpu_efficiency"] = efficiency(xr)
    if rank == 0 and world > 1:
        out["value_note"] = ("value = the sum over GPUs of independent, collective-free config-2 chunk reductions "
                             "(weak scaling); it is not the SURVEY 8(e) efficiency, which is per_gpu_efficiency")

    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
