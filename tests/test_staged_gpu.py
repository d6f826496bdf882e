"""GPU: host-staged chunk reduction (gloo_hip_reduce_staged) — a chunk in
pinned host memory reduced by the HIP kernel, zero-copy (piece 0) or staged
through device scratch — in one pass when the chunk fits one piece, else
pipelined in pieces of at least 16 MiB (smaller requested pieces are raised
to 16 MiB) — bit for bit against the oracle restatement of gloo/math.h."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    t = pytest.importorskip("torch")
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.mark.parametrize("dtype,op,n,piece", [
    ("f32", "sum", 1 << 20, 0),            # default: zero-copy (torch pins mapped memory)
    ("f32", "sum", 1_000_003, 65_537),     # below 16 MiB: one staged pass
    ("f32", "max", 4099, 1 << 20),         # one piece
    ("f32", "sum", 9_000_017, 1),          # raised to 16 MiB pieces: 16 + 16 + 2.3 MB, pipelined
    ("bf16", "max", 20_000_003, 12_000_000),  # 24 MB pieces: 24 + 16 MB
    ("i64", "product", 5_000_001, 3_000_000),  # 24 MB pieces: 24 + 16 MB
    ("bf16", "product", 300_007, 50_000),
    ("f16", "min", 123_457, 10_000),
    ("i64", "sum", 77_777, 4096),
    ("bf16", "max", 300_007, 0),           # zero-copy, 16-bit, ragged
    ("i64", "product", 77_777, 0),
])
def test_staged_matches_oracle(torch, dtype, op, n, piece):
    import gloo_amd
    code, npt = oracle.DTYPES[dtype]
    rng = np.random.default_rng(n)
    if dtype in ("f16", "bf16"):
        f = rng.uniform(0.5, 2.0, 2 * n).astype(np.float32)
        bits = (f.astype(np.float16).view(np.uint16) if dtype == "f16"
                else (f.view(np.uint32) >> 16).astype(np.uint16))
        a, b = bits[:n].copy(), bits[n:].copy()
    elif dtype == "i64":
        a, b = rng.integers(-1 << 40, 1 << 40, (2, n), dtype=np.int64)
    else:
        a, b = rng.standard_normal((2, n)).astype(npt)
    want = oracle.reduce3(op, dtype, a, b)
    tdt = {"f32": torch.float32, "i64": torch.int64, "f16": torch.int16, "bf16": torch.int16}[dtype]
    hd = torch.from_numpy(a.view(np.int16) if a.dtype == np.uint16 else a).pin_memory()
    hs = torch.from_numpy(b.view(np.int16) if b.dtype == np.uint16 else b).pin_memory()
    dd = torch.empty(n, dtype=tdt, device="cuda:0")
    ds = torch.empty(n, dtype=tdt, device="cuda:0")
    s = torch.cuda.current_stream()
    gloo_amd.reduce_staged(op, dtype, hd.data_ptr(), hs.data_ptr(), n, dd.data_ptr(), ds.data_ptr(), piece,
                           s.cuda_stream)
    s.synchronize()
    got = hd.numpy().view(npt)
    assert (got.view(np.uint8) == want.view(np.uint8)).all()
    # the source chunk is left untouched
    assert (hs.numpy().view(npt).view(np.uint8) == b.view(np.uint8)).all()
