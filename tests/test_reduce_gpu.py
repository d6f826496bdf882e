"""GPU parity: the HIP kernels behind the C-ABI vs the reference's results.

Every comparison is bit-exact (integers, bytes and IEEE floats alike: the op
is one IEEE operation per element, no contraction, denormals preserved),
NaN payloads included: 16-bit SUM / PRODUCT emit the reference's NaN bits
(F16C's operand / 0xFE00 rule, c10's 0x7FC0), pinned by the "f16_nan" /
"bf16_nan" goldens.  The one documented exception is fp16 MAX / MIN at a NaN
or a pair of zeros, where the reference's F16C host body and its CUDA twin
disagree and the kernel follows the CUDA twin (`expected`).
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

DTYPES = list(oracle.DTYPES)
OPS = list(oracle.OPS)


@pytest.fixture(scope="module")
def hip():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gloo_amd
    return gloo_amd


def to_dev(arr, byte_offset=0, pad=64):
    """Copy a numpy array into fresh device memory at `byte_offset` from a
    256-B aligned allocation; returns (tensor, device pointer)."""
    import torch
    raw = np.frombuffer(np.ascontiguousarray(arr).tobytes(), dtype=np.uint8)
    t = torch.zeros(raw.size + byte_offset + pad, dtype=torch.uint8, device="cuda")
    if raw.size:
        t[byte_offset:byte_offset + raw.size].copy_(torch.from_numpy(raw.copy()))
    return t, t.data_ptr() + byte_offset


def from_dev(t, byte_offset, nbytes, npt):
    import torch
    torch.cuda.synchronize()
    return t[byte_offset:byte_offset + nbytes].cpu().numpy().view(npt).copy()


def assert_same(dtype, op, got, want):
    n = len(want)
    g = got.view(np.uint8).reshape(n, -1)
    w = want.view(np.uint8).reshape(n, -1)
    eq = (g == w).all(1)
    bad = np.where(~eq)[0]
    assert bad.size == 0, f"{dtype}/{op}: {bad.size} mismatches, first {bad[:5]}: got {got[bad[:5]]} want {want[bad[:5]]}"


def run3(hip, op, dtype, a, b, offs=(0, 0, 0), inplace=False):
    code, npt = oracle.DTYPES[dtype]
    n = len(a)
    nbytes = a.nbytes
    ta, pa = to_dev(a, offs[1])
    tb, pb = to_dev(b, offs[2])
    if inplace:
        hip.reduce_ptr(op, dtype, pa, pb, n)
        return from_dev(ta, offs[1], nbytes, npt)
    tc, pc = to_dev(np.zeros_like(a), offs[0])
    hip.reduce3_ptr(op, dtype, pc, pa, pb, n)
    return from_dev(tc, offs[0], nbytes, npt)


def expected(golden, dtype, op, a, b, key=None):
    """Reference golden except where the reference's F16C host specialisation
    and its CUDA kernel disagree (fp16 max/min with a NaN or two zeros): there
    the CUDA-kernel rule restated by the oracle."""
    want = golden[f"{key or dtype}/{op}"].copy()
    if dtype == "f16" and op in ("max", "min"):
        o = oracle.reduce3(op, dtype, a, b)
        fn = lambda x: ((x & 0x7C00) == 0x7C00) & ((x & 0x3FF) != 0)  # noqa: E731
        z = lambda x: (x & 0x7FFF) == 0  # noqa: E731
        m = fn(a) | fn(b) | (z(a) & z(b))
        want[m] = o[m]
    return want


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("op", OPS)
def test_golden_reduce3(hip, golden_math, dtype, op):
    a, b = golden_math[f"{dtype}/a"], golden_math[f"{dtype}/b"]
    got = run3(hip, op, dtype, a, b)
    assert_same(dtype, op, got, expected(golden_math, dtype, op, a, b))


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("op", OPS)
def test_golden_inplace(hip, golden_math, dtype, op):
    """The form every schedule calls: fn_->call(dst, src, n) = dst op= src."""
    a, b = golden_math[f"{dtype}/a"], golden_math[f"{dtype}/b"]
    got = run3(hip, op, dtype, a, b, inplace=True)
    assert_same(dtype, op, got, expected(golden_math, dtype, op, a, b))


@pytest.mark.parametrize("key,dtype", [("f16_nan", "f16"), ("bf16_nan", "bf16")])
@pytest.mark.parametrize("op", OPS)
def test_golden_nan_payloads(hip, golden_math, key, dtype, op):
    """Every ordered pair of signed quiet / signalling NaNs and specials: the
    reference's NaN bits byte for byte, 3-operand and in place, also at a
    misaligned start (element-wise edges and 16-B body alike)."""
    a, b = golden_math[f"{key}/a"], golden_math[f"{key}/b"]
    want = expected(golden_math, dtype, op, a, b, key)
    assert_same(dtype, op, run3(hip, op, dtype, a, b), want)
    assert_same(dtype, op, run3(hip, op, dtype, a, b, inplace=True), want)
    assert_same(dtype, op, run3(hip, op, dtype, a, b, offs=(2, 6, 10)), want)


def test_f16_scalar_defect_golden_not_reproduced(hip, golden_math):
    """The "f16_scalar_defect" golden: the reference's
    scalar float16 body returns a for a = 0x5359, b = 0x7532.  The kernel
    returns the round-to-nearest-even sum 0x7536, as the reference's F16C
    vector body and its CUDA twin do (test_oracle.py pins the golden)."""
    a, b = golden_math["f16_scalar_defect/a"], golden_math["f16_scalar_defect/b"]
    assert golden_math["f16_scalar_defect/sum"][0] == 0x5359
    for inplace in (False, True):
        got = run3(hip, "sum", "f16", a, b, inplace=inplace)
        assert got.view(np.uint16)[0] == 0x7536


def rand_inputs(dtype, n, rng):
    code, npt = oracle.DTYPES[dtype]
    if dtype in ("f32", "f64"):
        return rng.standard_normal(n).astype(npt)
    if dtype in ("f16", "bf16"):
        f = rng.standard_normal(n).astype(np.float32)
        if dtype == "f16":
            return f.astype(np.float16).view(np.uint16)
        return (f.view(np.uint32) >> 16).astype(np.uint16)
    return rng.integers(0, 256, n * np.dtype(npt).itemsize, dtype=np.uint8).view(npt)


@pytest.mark.parametrize("dtype", ["i8", "f16", "f32", "f64"])
def test_misaligned_offsets(hip, dtype):
    """Chunks start at arbitrary element offsets (gloo/allreduce_ring_chunked.h:128):
    every combination of destination / source misalignment inside 16 B."""
    rng = np.random.default_rng(11)
    code, npt = oracle.DTYPES[dtype]
    es = np.dtype(npt).itemsize
    for n in (1, 5, 33, 1000, 4099):
        a, b = rand_inputs(dtype, n, rng), rand_inputs(dtype, n, rng)
        want = oracle.reduce3("sum", dtype, a, b)
        for oc in range(0, 16, es):
            for ob in range(0, 16, es):
                oa = oc  # in-place: dst is a
                got = run3(hip, "sum", dtype, a, b, offs=(oc, oa, ob), inplace=True)
                assert_same(dtype, "sum", got, want)
        got = run3(hip, "max", dtype, a, b, offs=(4 % 16 // es * es, 0, 2 * es % 16))
        assert_same(dtype, "max", got, oracle.reduce3("max", dtype, a, b))


@pytest.mark.parametrize("n", [0, 1, 3, 4, 7, 255, 256, 257, 1023, 1024, 1025, 4095, 65537,
                               (1 << 20) + 13])
def test_sizes_f32_sum(hip, n):
    rng = np.random.default_rng(n)
    a, b = rand_inputs("f32", n, rng), rand_inputs("f32", n, rng)
    if n == 0:
        hip.reduce_ptr("sum", "f32", 0, 0, 0)
        return
    got = run3(hip, "sum", "f32", a, b, inplace=True)
    assert_same("f32", "sum", got, oracle.reduce3("sum", "f32", a, b))


@pytest.mark.parametrize("dtype", DTYPES)
def test_all_ops_ragged_sizes(hip, dtype):
    rng = np.random.default_rng(21)
    for n in (2, 17, 300, 5003):
        a, b = rand_inputs(dtype, n, rng), rand_inputs(dtype, n, rng)
        for op in OPS:
            got = run3(hip, op, dtype, a, b, offs=(0, 0, 0), inplace=True)
            assert_same(dtype, op, got, oracle.reduce3(op, dtype, a, b))


def test_nan_and_signed_zero_rules(hip):
    """max/min keep a NaN already in dst, ignore a NaN arriving in src, and keep
    dst on ties (-0 vs +0): `if (src op dst) dst = src` (gloo/cuda.cu:337-355)."""
    nan, inf = np.float32(np.nan), np.float32(np.inf)
    a = np.array([nan, 1.0, nan, -0.0, 0.0, -inf, 2.0], dtype=np.float32)
    b = np.array([1.0, nan, nan, 0.0, -0.0, inf, 2.0], dtype=np.float32)
    for op in ("max", "min"):
        got = run3(hip, op, "f32", a, b, inplace=True)
        want = oracle.reduce3(op, "f32", a, b)
        assert_same("f32", op, got, want)
        assert np.isnan(got[0]) and got[1] == 1.0 and np.signbit(got[3]) and not np.signbit(got[4])


def test_f32_denormals_preserved(hip):
    t = np.float32(1.17549435e-38)
    a = np.array([t / 4, -t / 8, t / 2, 1e-45], dtype=np.float32)
    b = np.array([t / 4, t / 16, -t / 4, 1e-45], dtype=np.float32)
    for op in ("sum", "product"):
        got = run3(hip, op, "f32", a, b)
        assert_same("f32", op, got, oracle.reduce3(op, "f32", a, b))


def test_integer_wrap(hip):
    a = np.array([127, -128, 100, -1], dtype=np.int8)
    b = np.array([1, -1, 100, -1], dtype=np.int8)
    for op in OPS:
        assert_same("i8", op, run3(hip, op, "i8", a, b), oracle.reduce3(op, "i8", a, b))
    a = np.array([2**63 - 1, -2**63, 3037000500], dtype=np.int64)
    b = np.array([1, -1, 3037000500], dtype=np.int64)
    for op in OPS:
        assert_same("i64", op, run3(hip, op, "i64", a, b), oracle.reduce3(op, "i64", a, b))


@pytest.mark.parametrize("k", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("dtype", ["f32", "bf16", "i32"])
def test_reduce_multi(hip, k, dtype):
    """Fused local multi-pointer fold (gloo/allreduce_local.cc:28-33)."""
    rng = np.random.default_rng(k)
    code, npt = oracle.DTYPES[dtype]
    n = 10007
    srcs = [rand_inputs(dtype, n, rng) for _ in range(k)]
    for off in (0, 4):
        bufs = [to_dev(s, off if j % 2 else 0) for j, s in enumerate(srcs)]
        tdst, pdst = to_dev(np.zeros_like(srcs[0]), 0)
        for op in OPS:
            hip.reduce_multi_ptr(op, dtype, pdst, [p for _, p in bufs], n)
            got = from_dev(tdst, 0, srcs[0].nbytes, npt)
            assert_same(dtype, op, got, oracle.reduce_multi(op, dtype, srcs))


def test_full_size_64mib_f32_sum_properties(hip):
    """BASELINE config 2 size (64 MiB fp32): bit-exact vs numpy's IEEE f32 add
    (== the oracle), and a + b - b round trip checked through the kernel."""
    import torch
    n = 16 * 1024 * 1024
    g = torch.Generator(device="cuda").manual_seed(1)
    a = torch.rand(n, device="cuda", generator=g) * 2 - 1
    b = torch.rand(n, device="cuda", generator=g) * 2 - 1
    ref = (a.cpu().numpy() + b.cpu().numpy())  # IEEE f32 add, element-wise
    c = torch.empty_like(a)
    hip.reduce3("sum", c, a, b)
    assert (c.cpu().numpy().view(np.uint32) == ref.view(np.uint32)).all()
    hip.reduce("sum", a, b)                     # in place, the schedules' form
    assert torch.equal(a, c)
    m = torch.empty_like(a)
    hip.reduce3("max", m, a, a)                 # idempotence
    assert torch.equal(m, a)


def test_stream_ordering(hip):
    """Launches are async on the caller's stream (gloo/cuda.h:326-333)."""
    import torch
    s = torch.cuda.Stream()
    n = 1 << 22
    a = torch.ones(n, device="cuda")
    b = torch.ones(n, device="cuda")
    with torch.cuda.stream(s):
        for _ in range(10):
            hip.reduce("sum", a, b)             # uses the current (side) stream
    s.synchronize()
    assert float(a[0]) == 11.0 and float(a[-1]) == 11.0


@pytest.mark.parametrize("dtype,inplace", [("u8", True), ("u8", False), ("i8", True)])
def test_beyond_4gi_elements(hip, dtype, inplace):
    """Maximum sizes: n = 2^32 + 4099 one-byte elements at a misaligned start.

    The reference's kernels index with `int n` (gloo/cuda.cu:274-401) and its
    ring-chunked `count`/`bytes_` are `int` (gloo/cuda_allreduce_ring_chunked.h:54-55),
    so nothing past 2^31 elements is reachable there; the C-ABI takes size_t.
    A constant fill catches any 32-bit offset wrap both ways: a wrapped in-place
    kernel would leave the high region at `x` and fold the low one twice.  Spot
    values near 2^31, 2^32 and the ragged tail are checked against the oracle.
    """
    import torch
    code, npt = oracle.DTYPES[dtype]
    n = (1 << 32) + 4099
    off = 3
    x, y = (7, 250) if dtype == "u8" else (-100, -90)
    ta = torch.full((n + off + 64,), x, dtype=torch.uint8 if dtype == "u8" else torch.int8, device="cuda")
    tb = torch.full_like(ta, y)
    spots = np.array([0, 1, (1 << 31) - 1, 1 << 31, (1 << 32) - 1, 1 << 32, n - 2, n - 1], dtype=np.int64)
    rng = np.random.default_rng(11)
    sa = rng.integers(-128 if dtype == "i8" else 0, 128 if dtype == "i8" else 256, spots.size).astype(npt)
    sb = rng.integers(-128 if dtype == "i8" else 0, 128 if dtype == "i8" else 256, spots.size).astype(npt)
    idx = torch.from_numpy(spots + off).cuda()
    ta[idx] = torch.from_numpy(sa).cuda()
    tb[idx] = torch.from_numpy(sb).cuda()
    pa, pb = ta.data_ptr() + off, tb.data_ptr() + off
    if inplace:
        hip.reduce_ptr("sum", dtype, pa, pb, n)
        out = ta
    else:
        out = torch.zeros_like(ta)
        hip.reduce3_ptr("sum", dtype, out.data_ptr() + off, pa, pb, n)
    torch.cuda.synchronize()
    body = out[off:off + n]
    want_fill = oracle.reduce3("sum", dtype, np.array([x], npt), np.array([y], npt))[0]
    eq = body == int(want_fill)
    eq[torch.from_numpy(spots).cuda()] = True
    assert bool(eq.all()), "32-bit offset wrap or missed region"
    del eq
    got = out[idx].cpu().numpy().view(npt)
    assert (got == oracle.reduce3("sum", dtype, sa, sb)).all()
    # guard bytes either side untouched
    if not inplace:
        assert bool((out[:off] == 0).all()) and bool((out[off + n:] == 0).all())
    else:
        assert bool((out[:off] == x).all()) and bool((out[off + n:] == x).all())
