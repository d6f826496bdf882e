"""Generate tests/golden/*.npz from the REFERENCE itself.  TEST INFRASTRUCTURE.

Runs only where /root/reference exists (this build container): it calls
oracle/_ref/libgloo_ref.so, which oracle/Makefile compiles from the unmodified
reference sources, and records inputs + reference outputs as data fixtures.
The fixtures (not the reference) travel to the GPU box.

  math_golden.npz      gloo::sum/product/max/min<T>(c, a, b, n), gloo/math.h:15-73,
                       every dtype of include/gloo_amd.h, n = 4099, inputs with
                       zeros / infs / NaNs / denormals sprinkled in.  fp16 via the
                       F16C body (gloo/math.cc:17-97); bf16 via c10::BFloat16.
  sched_golden.npz     AllreduceRingChunked / AllreduceHalvingDoubling /
                       AllreduceRing / ReduceScatterHalvingDoubling outputs at
                       P ranks (threads over the reference's TCP transport).
  bcube_golden.npz     AllreduceBcube (gloo/allreduce_bcube.h) on contexts of
                       base 2, 3 and 4: the P = base^k grid of
                       gloo/test/allreduce_test.cc:271-299 plus larger counts,
                       several pointers, other dtypes and ops, and two P that
                       are not powers of the base (the reference's ranges as
                       they fall there); every rank's output is kept.

Usage:  make -C oracle ref && python oracle/gen_golden.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
SEED = 20240601

ALGOS = {"ring_chunked": 0, "halving_doubling": 1, "ring": 2, "local": 3}


def special_floats(npt):
    f = np.finfo(npt)
    return np.array([0.0, -0.0, np.inf, -np.inf, np.nan, f.tiny / 4, -f.tiny / 8, f.max,
                     -f.max, 1.0, -1.0], dtype=npt)


def make_inputs(dtype, n, rng):
    code, npt = oracle.DTYPES[dtype]
    if dtype in ("f32", "f64"):
        x = (rng.standard_normal(n) * np.where(rng.random(n) < 0.5, 1.0, 1e-3)).astype(npt)
        sp = special_floats(npt)
        idx = rng.integers(0, n, n // 40)
        x[idx] = sp[rng.integers(0, len(sp), len(idx))]
        return x
    if dtype in ("f16", "bf16"):
        # random finite values of a sane range plus special encodings
        f = (rng.standard_normal(n) * 4).astype(np.float32)
        conv = oracle.lib().oracle_f32_to_f16 if dtype == "f16" else oracle.lib().oracle_f32_to_bf16
        x = np.array([conv(float(v)) for v in f], dtype=np.uint16)
        if dtype == "f16":
            sp = np.array([0x0000, 0x8000, 0x7C00, 0xFC00, 0x7E00, 0x0001, 0x83FF, 0x7BFF, 0xFBFF,
                           0x3C00, 0xBC00], dtype=np.uint16)
        else:
            sp = np.array([0x0000, 0x8000, 0x7F80, 0xFF80, 0x7FC0, 0x0001, 0x807F, 0x7F7F, 0xFF7F,
                           0x3F80, 0xBF80], dtype=np.uint16)
        idx = rng.integers(0, n, n // 40)
        x[idx] = sp[rng.integers(0, len(sp), len(idx))]
        return x
    return rng.integers(0, 256, n * np.dtype(npt).itemsize, dtype=np.uint8).view(npt)


def gen_math():
    rng = np.random.default_rng(SEED)
    n = 4099
    out = {}
    for dtype in oracle.DTYPES:
        a = make_inputs(dtype, n, rng)
        b = make_inputs(dtype, n, rng)
        out[f"{dtype}/a"] = a
        out[f"{dtype}/b"] = b
        for op in oracle.OPS:
            out[f"{dtype}/{op}"] = oracle.ref_reduce3(op, dtype, a, b)
    # App. A.1: the scalar float16 path as shipped without GLOO_USE_AVX.
    a = np.array([0x5359], dtype=np.uint16)
    b = np.array([0x7532], dtype=np.uint16)
    c = np.empty_like(a)
    oracle.ref().ref_reduce3_f16_scalar(1, c.ctypes.data, a.ctypes.data, b.ctypes.data, 1)
    out["f16_scalar_defect/a"], out["f16_scalar_defect/b"], out["f16_scalar_defect/sum"] = a, b, c
    out.update(nan_pairs())
    np.savez_compressed(os.path.join(OUT, "math_golden.npz"), **out)
    print("math_golden.npz:", len(out), "arrays")


def nan_pairs():
    """Every ordered pair of 16-bit NaNs (signed, quiet and signalling payloads)
    and specials, for the NaN bits of SUM / PRODUCT: the F16C body keeps the
    second operand's payload, else the first's, else emits 0xFE00; c10's bf16
    emits 0x7FC0.  The length is a multiple of 8, so every element goes through
    the F16C body (gloo/math.cc:27-32), none through the scalar leftovers."""
    f16 = [0x7E00, 0xFE00, 0x7C01, 0x7D55, 0xFD55, 0x7FFF, 0xFC01, 0x3C00, 0x7C00, 0xFC00,
           0x0000, 0x8000, 0x0001, 0x7BFF]
    bf16 = [0x7FC0, 0xFFC0, 0x7F81, 0x7FD5, 0xFFD5, 0x7FFF, 0xFF81, 0x3F80, 0x7F80, 0xFF80,
            0x0000, 0x8000, 0x0001, 0x7F7F]
    out = {}
    for dtype, vals in (("f16", f16), ("bf16", bf16)):
        v = np.array(vals, dtype=np.uint16)
        a = np.repeat(v, len(v))
        b = np.tile(v, len(v))
        pad = (-len(a)) % 8
        a = np.concatenate([a, np.full(pad, v[-1], np.uint16)])
        b = np.concatenate([b, np.full(pad, v[-1], np.uint16)])
        out[f"{dtype}_nan/a"], out[f"{dtype}_nan/b"] = a, b
        for op in oracle.OPS:
            out[f"{dtype}_nan/{op}"] = oracle.ref_reduce3(op, dtype, a, b)
    return out


def ref_allreduce(algo, op, dtype, inputs):
    code, npt = oracle.DTYPES[dtype]
    P, k, n = inputs.shape
    out = np.empty_like(inputs)
    rc = oracle.ref().ref_allreduce(ALGOS[algo], oracle.OPS[op], code, P, k, n,
                                    inputs.ctypes.data, out.ctypes.data)
    if rc:
        raise RuntimeError(f"ref_allreduce({algo},{P},{n}) = {rc}: {oracle.ref().ref_last_error()}")
    return out


def ref_reduce_scatter(op, dtype, inputs, recv):
    code, npt = oracle.DTYPES[dtype]
    P, n = inputs.shape
    out = np.empty_like(inputs)
    recv = np.ascontiguousarray(recv, dtype=np.int32)
    rc = oracle.ref().ref_reduce_scatter(oracle.OPS[op], code, P, n, recv.ctypes.data,
                                         inputs.ctypes.data, out.ctypes.data)
    if rc:
        raise RuntimeError(f"ref_reduce_scatter({P},{n}) = {rc}: {oracle.ref().ref_last_error()}")
    return out


def even_recv(P, n):
    """recvElems exactly as gloo/test/reduce_scatter_test.cc:86-92 builds them."""
    out, rem, chunk = [], n, (n + P - 1) // P
    for _ in range(P):
        out.append(min(chunk, rem))
        rem = rem - chunk if rem > chunk else 0
    return np.array(out, dtype=np.int32)


def sched_inputs(dtype, op, shape, rng):
    code, npt = oracle.DTYPES[dtype]
    if op == "product":
        f = rng.uniform(0.5, 2.0, shape).astype(np.float32)
    else:
        f = rng.standard_normal(shape).astype(np.float32)
    if dtype == "f32":
        return f
    if dtype == "f64":
        return f.astype(np.float64)
    conv = oracle.lib().oracle_f32_to_f16 if dtype == "f16" else oracle.lib().oracle_f32_to_bf16
    return np.vectorize(lambda v: conv(float(v)), otypes=[np.uint16])(f)


def gen_sched():
    rng = np.random.default_rng(SEED + 1)
    out = {}
    cases = []
    for P in (1, 2, 3, 5, 8):
        for n in (1, 1000) + ((10007,) if P in (3, 8) else ()):
            cases.append(("ring_chunked", "sum", "f32", P, 1, n))
    cases += [("ring_chunked", "sum", "f32", 3, 2, 1000), ("ring_chunked", "max", "f32", 5, 1, 999),
              ("ring_chunked", "sum", "f64", 4, 1, 4099), ("ring_chunked", "product", "f32", 3, 1, 777)]
    for P in (1, 2, 3, 5, 6, 8):
        for n in (1, 64, 1000) + ((10007,) if P in (5, 8) else ()):
            cases.append(("halving_doubling", "sum", "f32", P, 1, n))
    cases += [("halving_doubling", "min", "f32", 5, 1, 1000), ("halving_doubling", "sum", "f32", 3, 3, 500),
              ("halving_doubling", "sum", "f64", 7, 1, 3001)]
    cases += [("ring", "sum", "f32", 3, 1, 1000), ("ring", "sum", "f32", 8, 1, 4096),
              ("local", "sum", "f32", 1, 4, 1000)]
    for algo, op, dtype, P, k, n in cases:
        x = sched_inputs(dtype, op, (P, k, n), rng)
        y = ref_allreduce(algo, op, dtype, x)
        key = f"{algo}/{op}/{dtype}/P{P}/k{k}/n{n}"
        out[key + "/in"] = x
        if algo == "ring":
            # AllreduceRing folds in a rank-dependent order
            # (gloo/allreduce_ring.h:80-90): ranks differ in the last bits.
            out[key + "/out"] = y[:, 0].copy()
        else:
            # every rank and pointer ends with the same bytes; keep one copy
            assert all((y[r, j].view(np.uint8) == y[0, 0].view(np.uint8)).all()
                       for r in range(P) for j in range(k)), key
            out[key + "/out"] = y[0, 0].copy()
    rs_cases = []
    for P in (1, 2, 3, 5, 8):
        for n in (100,) + ((10007,) if P in (3, 8) else ()):
            rs_cases.append(("sum", "f32", P, n))
    for dtype in ("f16", "bf16"):
        for op in ("sum", "product", "max", "min"):
            rs_cases.append((op, dtype, 8, 4096))
    rs_cases.append(("sum", "f16", 4, 1024))  # gloo/test/reduce_scatter_test.cc HalfPrecisionTest shape
    for op, dtype, P, n in rs_cases:
        x = sched_inputs(dtype, op, (P, n), rng)
        recv = even_recv(P, n)
        y = ref_reduce_scatter(op, dtype, x, recv)
        key = f"reduce_scatter/{op}/{dtype}/P{P}/n{n}"
        out[key + "/in"] = x
        out[key + "/recv"] = recv
        # only rank r's reduced block out[r, :recv[r]] is defined; concatenate
        out[key + "/out"] = np.concatenate([y[r, :recv[r]] for r in range(P)])
    # New-style gloo::allreduce(opts), ring (gloo/allreduce.cc:147-392).
    new_cases = []
    for P in (2, 3, 5, 8):
        for n in (1, 1000, 4099):
            new_cases.append(("sum", "f32", P, 0, 1, n, 0))
    new_cases += [("sum", "f32", 3, 1, 1, 1000, 128), ("sum", "f32", 3, 3, 2, 1000, 128),
                  ("sum", "f32", 4, 2, 1, 4099, 256), ("sum", "f32", 5, 0, 3, 777, 100),
                  ("max", "f32", 4, 0, 1, 3000, 128), ("sum", "bf16", 4, 2, 2, 2000, 256),
                  ("sum", "u64", 4, 0, 1, 1000, 128), ("product", "f64", 3, 2, 1, 999, 64)]
    for op, dtype, P, nin, nout, n, seg in new_cases:
        x = sched_inputs(dtype, op, (P, max(nin, 1), n), rng) if dtype not in ("u64",) else \
            rng.integers(0, 1 << 40, (P, max(nin, 1), n), dtype=np.uint64)
        init = sched_inputs(dtype, op, (P, nout, n), rng) if dtype not in ("u64",) else \
            rng.integers(0, 1 << 40, (P, nout, n), dtype=np.uint64)
        code, npt = oracle.DTYPES[dtype]
        y = np.ascontiguousarray(init.copy())
        xin = np.ascontiguousarray(x[:, :nin]) if nin else np.zeros(1, dtype=npt)
        rc = oracle.ref().ref_allreduce_new(oracle.OPS[op], code, P, nin, nout, n, seg,
                                            xin.ctypes.data, y.ctypes.data)
        if rc:
            raise RuntimeError(f"ref_allreduce_new failed {rc}: {oracle.ref().ref_last_error()}")
        key = f"allreduce_new/{op}/{dtype}/P{P}/i{nin}/o{nout}/n{n}/s{seg}"
        assert all((y[r, j].view(np.uint8) == y[0, 0].view(np.uint8)).all()
                   for r in range(P) for j in range(nout)), key
        if nin:
            out[key + "/in"] = x[:, :nin]
        out[key + "/init"] = init
        out[key + "/out"] = y[0, 0].copy()
    np.savez_compressed(os.path.join(OUT, "sched_golden.npz"), **out)
    print("sched_golden.npz:", len(out), "arrays")


def ref_allreduce_bcube(op, dtype, base, inputs):
    code, npt = oracle.DTYPES[dtype]
    P, k, n = inputs.shape
    out = np.empty_like(inputs)
    rc = oracle.ref().ref_allreduce_bcube(oracle.OPS[op], code, P, base, k, n, inputs.ctypes.data,
                                          out.ctypes.data)
    if rc:
        raise RuntimeError(f"ref_allreduce_bcube({P},{base},{n}) = {rc}: {oracle.ref().ref_last_error()}")
    return out


def bcube_cases():
    """(op, dtype, P, base, k, n): the reference's own grid first."""
    cases = []
    for base, Ps in ((2, (2, 4, 8, 16)), (3, (3, 9, 27)), (4, (4, 16))):
        for P in Ps:
            for n in (1, 64, 1000):
                cases.append(("sum", "f32", P, base, 1, n))
    cases += [("sum", "f32", 8, 2, 1, 20011), ("sum", "f32", 9, 3, 1, 4099), ("sum", "f32", 4, 2, 3, 1000),
              ("max", "f32", 8, 2, 1, 4099), ("min", "f32", 4, 4, 1, 777), ("product", "f64", 4, 2, 2, 999),
              ("sum", "bf16", 8, 2, 1, 2000), ("sum", "f16", 9, 3, 1, 1001), ("sum", "i32", 4, 2, 1, 3000),
              # P not a power of the base: the reference's ranges as they fall
              ("sum", "f32", 6, 2, 1, 1000), ("sum", "f32", 5, 3, 1, 500)]
    return cases


def gen_bcube():
    rng = np.random.default_rng(SEED + 3)
    out = {}
    for op, dtype, P, base, k, n in bcube_cases():
        x = _values(dtype, op, (P, k, n), rng)
        y = ref_allreduce_bcube(op, dtype, base, np.ascontiguousarray(x))
        key = f"bcube/{op}/{dtype}/P{P}/b{base}/k{k}/n{n}"
        for r in range(P):  # each rank's pointers end alike (the local broadcast)
            assert all((y[r, j].view(np.uint8) == y[r, 0].view(np.uint8)).all() for j in range(k)), key
        out[key + "/in"] = x
        out[key + "/out"] = y[:, 0].copy()  # [P][n]: every rank's result
    np.savez_compressed(os.path.join(OUT, "bcube_golden.npz"), **out)
    print("bcube_golden.npz:", len(out), "arrays")


def _values(dtype, op, shape, rng):
    if dtype in ("u64", "i32"):
        npt = oracle.DTYPES[dtype][1]
        hi = 1 << 40 if dtype == "u64" else 1 << 20
        return rng.integers(0, hi, shape, dtype=np.int64).astype(npt)
    return sched_inputs(dtype, op, shape, rng)


def gen_newstyle():
    """newstyle_golden.npz: gloo::allreduce(opts) with BCUBE
    (gloo/allreduce.cc:397-669) and gloo::reduce(opts) (gloo/reduce.cc:21-247)."""
    rng = np.random.default_rng(SEED + 2)
    out = {}
    bcube = []
    for P in (2, 3, 4, 5, 6, 7, 8, 12):
        for n in (1, 10, 1000, 4099):
            bcube.append(("sum", "f32", P, 0, 1, n))
    bcube += [("sum", "f32", 4, 2, 1, 1000), ("sum", "f32", 6, 3, 2, 999), ("sum", "f32", 8, 1, 3, 4099),
              ("max", "f32", 6, 0, 1, 3000), ("min", "f32", 8, 0, 2, 777), ("product", "f64", 3, 2, 1, 999),
              ("sum", "bf16", 8, 0, 1, 4096), ("sum", "f16", 4, 0, 1, 1024), ("sum", "u64", 7, 2, 2, 1000),
              ("max", "bf16", 12, 0, 1, 5000)]
    for op, dtype, P, nin, nout, n in bcube:
        code, npt = oracle.DTYPES[dtype]
        x = _values(dtype, op, (P, max(nin, 1), n), rng)
        init = _values(dtype, op, (P, nout, n), rng)
        y = np.ascontiguousarray(init.copy())
        xin = np.ascontiguousarray(x[:, :nin]) if nin else np.zeros(1, dtype=npt)
        rc = oracle.ref().ref_allreduce_new_algo(2, oracle.OPS[op], code, P, nin, nout, n, 0,
                                                 xin.ctypes.data, y.ctypes.data)
        if rc:
            raise RuntimeError(f"bcube failed {rc}: {oracle.ref().ref_last_error()}")
        key = f"bcube/{op}/{dtype}/P{P}/i{nin}/o{nout}/n{n}/s0"
        assert all((y[r, j].view(np.uint8) == y[0, 0].view(np.uint8)).all()
                   for r in range(P) for j in range(nout)), key
        if nin:
            out[key + "/in"] = x[:, :nin]
        out[key + "/init"] = init
        out[key + "/out"] = y[0, 0].copy()
    red = []
    for P in (2, 3, 4, 7):
        for n in (1, 10, 1000, 10000):
            red.append(("sum", "f32", P, 0, n, P - 1, 128 if n >= 1000 else 0))
    red += [("sum", "f32", 4, 1, 1000, 0, 128), ("sum", "f32", 5, 1, 4099, 2, 0), ("max", "f32", 3, 0, 999, 1, 64),
            ("product", "f64", 4, 1, 777, 3, 0), ("sum", "bf16", 8, 1, 4096, 5, 256), ("min", "f16", 6, 0, 2000, 0, 0),
            ("sum", "u64", 7, 1, 1000, 6, 128), ("sum", "f32", 8, 0, 20011, 3, 0)]
    for op, dtype, P, has_in, n, root, seg in red:
        code, npt = oracle.DTYPES[dtype]
        x = _values(dtype, op, (P, n), rng)
        init = _values(dtype, op, (P, n), rng)
        y = np.ascontiguousarray(init.copy())
        xin = np.ascontiguousarray(x) if has_in else np.zeros(1, dtype=npt)
        rc = oracle.ref().ref_reduce_new(oracle.OPS[op], code, P, has_in, n, seg, root,
                                         xin.ctypes.data, y.ctypes.data)
        if rc:
            raise RuntimeError(f"reduce failed {rc}: {oracle.ref().ref_last_error()}")
        key = f"reduce/{op}/{dtype}/P{P}/i{has_in}/n{n}/r{root}/s{seg}"
        if has_in:
            out[key + "/in"] = x[:, None, :]
        out[key + "/init"] = init[:, None, :]
        out[key + "/out"] = y  # every rank's output buffer, [P][n]
    np.savez_compressed(os.path.join(OUT, "newstyle_golden.npz"), **out)
    print("newstyle_golden.npz:", len(out), "arrays")


def gen_bw():
    """bw_golden.json + bw_golden.npz: the reference's outputs in the
    bandwidth regime of BASELINE configs 3-5 and at the reference's large-P
    test grid (gloo/test/allreduce_test.cc:261-269,
    gloo/test/reduce_scatter_test.cc:79-196).

    The big cases keep only seed + per-rank SHA-256 digest + sampled values
    (tests/bw_inputs.py draws the inputs identically on the GPU box); the
    large-P cases are small and keep whole arrays."""
    import json
    import time
    sys.path.insert(0, os.path.join(os.path.dirname(OUT)))
    import bw_inputs as bw
    seed = SEED + 3
    big = [("ring_chunked", "sum", "f32", 8, 1 << 26),        # config 3: 256 MiB per rank
           ("halving_doubling", "sum", "f32", 8, 1 << 22),    # config 4, 16 MiB per rank
           ("halving_doubling", "sum", "f32", 8, 5000011),    # ragged: misaligned chunk offsets
           ("ring_chunked", "max", "f32", 8, 10000019)]
    big += [("reduce_scatter", op, dt, 8, 1 << 20) for dt in ("f16", "bf16")
            for op in ("sum", "product", "max", "min")]          # config 5
    big += [("reduce_scatter", "sum", "f32", 8, 1000003)]
    cases = []
    for i, (algo, op, dtype, P, n) in enumerate(big):
        t0 = time.time()
        cs = seed + i
        x = np.stack([bw.make_input(dtype, op, n, cs, r) for r in range(P)])
        key = f"{algo}/{op}/{dtype}/P{P}/n{n}"
        if algo == "reduce_scatter":
            recv = bw.even_recv(P, n)
            y = ref_reduce_scatter(op, dtype, x, np.array(recv, np.int32))
            outs = [y[r, :recv[r]] for r in range(P)]
        else:
            recv = None
            y = ref_allreduce(algo, op, dtype, x[:, None, :])[:, 0]
            outs = [y[r] for r in range(P)]
            assert all((o.view(np.uint8) == outs[0].view(np.uint8)).all() for o in outs), key
        samples = []
        for r in range(P):
            idx = bw.sample_index(len(outs[r]))
            samples.append({"idx": idx.tolist(), "val": outs[r][idx].view(
                np.uint32 if outs[r].dtype.itemsize == 4 else np.uint16).tolist()})
        cases.append({"key": key, "algo": algo, "op": op, "dtype": dtype, "P": P, "n": n, "seed": cs,
                      "recv": recv, "digests": [bw.digest(o) for o in outs], "samples": samples})
        print(f"bw {key}: {time.time() - t0:.1f} s", flush=True)
        del x, y, outs
    with open(os.path.join(OUT, "bw_golden.json"), "w") as f:
        json.dump({"generator": "oracle/gen_golden.py bw (reference: oracle/_ref/libgloo_ref.so)",
                   "inputs": "tests/bw_inputs.py make_input(dtype, op, n, seed, rank)",
                   "cases": cases}, f, indent=0)
    # large P: the reference's own test grid beyond the mesh range (P > 8)
    rng = np.random.default_rng(seed + 100)
    out = {}
    for P in (9, 13, 16, 24, 32):
        for n in (1, 64, 1000):
            x = sched_inputs("f32", "sum", (P, 1, n), rng)
            y = ref_allreduce("halving_doubling", "sum", "f32", x)
            assert all((y[r, 0].view(np.uint8) == y[0, 0].view(np.uint8)).all() for r in range(P))
            key = f"halving_doubling/sum/f32/P{P}/k1/n{n}"
            out[key + "/in"], out[key + "/out"] = x, y[0, 0].copy()
    for P in (9, 13, 16, 24, 32):
        for n in (100, 1000):
            x = sched_inputs("f32", "sum", (P, n), rng)
            recv = even_recv(P, n)
            y = ref_reduce_scatter("sum", "f32", x, recv)
            key = f"reduce_scatter/sum/f32/P{P}/n{n}"
            out[key + "/in"], out[key + "/recv"] = x, recv
            out[key + "/out"] = np.concatenate([y[r, :recv[r]] for r in range(P)])
    x = sched_inputs("f16", "max", (16, 1000), rng)
    recv = even_recv(16, 1000)
    y = ref_reduce_scatter("max", "f16", x, recv)
    out["reduce_scatter/max/f16/P16/n1000/in"], out["reduce_scatter/max/f16/P16/n1000/recv"] = x, recv
    out["reduce_scatter/max/f16/P16/n1000/out"] = np.concatenate([y[r, :recv[r]] for r in range(16)])
    np.savez_compressed(os.path.join(OUT, "bw_golden.npz"), **out)
    print("bw_golden.json:", len(cases), "cases; bw_golden.npz:", len(out), "arrays")


def gen_bw_extend():
    """Append to bw_golden.json the largest BASELINE sizes:
    config 5 at 16 Mi and 64 Mi elements per rank, config 4 at 256 MiB per
    rank.  Existing cases are kept as they are; a key already present is
    skipped, so the step is idempotent."""
    import json
    import time
    sys.path.insert(0, os.path.join(os.path.dirname(OUT)))
    import bw_inputs as bw
    path = os.path.join(OUT, "bw_golden.json")
    doc = json.load(open(path))
    have = {c["key"] for c in doc["cases"]}
    seed = SEED + 50
    extra = [("reduce_scatter", "sum", "f16", 8, 1 << 24), ("reduce_scatter", "max", "bf16", 8, 1 << 24),
             ("reduce_scatter", "product", "bf16", 8, 1 << 26), ("reduce_scatter", "sum", "f16", 8, 1 << 26),
             ("halving_doubling", "sum", "f32", 8, 1 << 26),
             # the top of the config-4 sweep: 1 GiB per rank
             ("halving_doubling", "sum", "f32", 8, 1 << 28),
             # the same per-rank size at 4 ranks: 4 rank processes fit one GPU's queues, so the
             # one-GPU tests run the mesh route at 1 GiB per rank too
             ("halving_doubling", "sum", "f32", 4, 1 << 28)]
    for i, (algo, op, dtype, P, n) in enumerate(extra):
        key = f"{algo}/{op}/{dtype}/P{P}/n{n}"
        if key in have:
            continue
        t0 = time.time()
        cs = seed + i
        x = np.stack([bw.make_input(dtype, op, n, cs, r) for r in range(P)])
        if algo == "reduce_scatter":
            recv = bw.even_recv(P, n)
            y = ref_reduce_scatter(op, dtype, x, np.array(recv, np.int32))
            outs = [y[r, :recv[r]] for r in range(P)]
        else:
            recv = None
            y = ref_allreduce(algo, op, dtype, x[:, None, :])[:, 0]
            outs = [y[r] for r in range(P)]
            assert all((o.view(np.uint8) == outs[0].view(np.uint8)).all() for o in outs), key
        samples = []
        for r in range(P):
            idx = bw.sample_index(len(outs[r]))
            samples.append({"idx": idx.tolist(), "val": outs[r][idx].view(
                np.uint32 if outs[r].dtype.itemsize == 4 else np.uint16).tolist()})
        doc["cases"].append({"key": key, "algo": algo, "op": op, "dtype": dtype, "P": P, "n": n, "seed": cs,
                             "recv": recv, "digests": [bw.digest(o) for o in outs], "samples": samples})
        print(f"bw+ {key}: {time.time() - t0:.1f} s", flush=True)
        del x, y, outs
    with open(path, "w") as f:
        json.dump(doc, f, indent=0)


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    which = sys.argv[1:] or ["math", "sched", "newstyle"]
    if "bw" in which:
        gen_bw()
    if "bw_extend" in which:
        gen_bw_extend()
    if "math" in which:
        gen_math()
    if "sched" in which:
        gen_sched()
    if "newstyle" in which:
        gen_newstyle()
    if "bcube" in which:
        gen_bcube()
