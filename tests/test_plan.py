"""CPU: the C++ schedule planners (gloo_amd/csrc/plan.cc) reproduce the
reference's allreduce / reduce-scatter schedules bit for bit.

tests/golden/sched_golden.npz holds outputs of the reference's own
AllreduceRingChunked / AllreduceHalvingDoubling / AllreduceRing /
AllreduceLocal / ReduceScatterHalvingDoubling (oracle/gen_golden.py, ranks as
threads over the reference's TCP transport).  Here all ranks' plans are
executed by tests/plan_sim.py with the oracle reduction, under several random
interleavings, and compared byte for byte.
"""
import numpy as np
import pytest

from plan_sim import ProtocolError, get_plan, simulate

import oracle


def golden_cases(g):
    keys = sorted({k.rsplit("/", 1)[0] for k in g.files})
    return keys


def _keys():
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "sched_golden.npz"))
    return golden_cases(z)


@pytest.mark.parametrize("case", _keys())
def test_plan_matches_reference_golden(golden_sched, case):
    parts = case.split("/")
    algo, op, dtype = parts[0], parts[1], parts[2]
    x = golden_sched[case + "/in"] if case + "/in" in golden_sched.files else None
    want = golden_sched[case + "/out"]
    for seed in (0, 1, 2):
        if algo == "allreduce_new":
            nin = int(parts[4][1:])
            seg = int(parts[7][1:])
            init = golden_sched[case + "/init"]
            ins = golden_sched[case + "/in"] if nin else None
            y = simulate(algo, op, dtype, init, seed=seed, ins=ins, max_seg=seg)
            for r in range(y.shape[0]):
                for j in range(y.shape[1]):
                    assert (y[r, j].view(np.uint8) == want.view(np.uint8)).all(), (r, j)
            got = y[0, 0]
        elif algo == "reduce_scatter":
            recv = golden_sched[case + "/recv"]
            y = simulate(algo, op, dtype, x[:, None, :], recv=recv, seed=seed)
            got = np.concatenate([y[r, 0, :recv[r]] for r in range(len(recv))])
        elif algo == "ring":
            y = simulate(algo, op, dtype, x, seed=seed)
            got = y[:, 0]
        else:
            y = simulate(algo, op, dtype, x, seed=seed)
            P, k = y.shape[:2]
            for r in range(P):
                for j in range(k):
                    assert (y[r, j].view(np.uint8) == y[0, 0].view(np.uint8)).all()
            got = y[0, 0]
        assert got.shape == want.shape
        bad = np.where(~(got.view(np.uint8).reshape(len(got.reshape(-1)), -1) ==
                         want.view(np.uint8).reshape(len(want.reshape(-1)), -1)).all(1))[0]
        assert bad.size == 0, f"{case} seed {seed}: {bad.size} mismatches, first {bad[:5]}"


@pytest.mark.parametrize("algo", ["ring_chunked", "halving_doubling", "ring"])
@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 6, 7, 8, 9, 13, 16])
@pytest.mark.parametrize("n", [0, 1, 4, 100, 1000])
def test_allreduce_grid_closed_form(algo, P, n):
    """The reference test grid (gloo/test/allreduce_test.cc:241-269) with its
    closed-form fixture (gloo/test/base_test.h:184-236): src[j] = j*P + rank,
    sum over ranks = j*P*P + P*(P-1)/2."""
    if algo == "ring" and P > 9:
        pytest.skip("plain ring grid stops at 9 in this sweep")
    x = np.array([[np.arange(n, dtype=np.float64) * P + r] for r in range(P)], dtype=np.float64)
    y = simulate(algo, "sum", "f64", x, seed=P * 31 + n)
    want = np.arange(n, dtype=np.float64) * P * P + P * (P - 1) / 2
    for r in range(P):
        assert (y[r, 0] == want).all()


@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 6, 7, 8, 9, 13, 16, 24, 32])
@pytest.mark.parametrize("n", [4, 100, 1000])
def test_reduce_scatter_grid(P, n):
    """gloo/test/reduce_scatter_test.cc:79-105 grid: every rank holds its rank,
    rank r's block equals P(P-1)/2."""
    chunk = (n + P - 1) // P
    recv, rem = [], n
    for _ in range(P):
        recv.append(min(chunk, rem))
        rem = rem - chunk if rem > chunk else 0
    x = np.array([[np.full(n, r, dtype=np.float32)] for r in range(P)])
    y = simulate("reduce_scatter", "sum", "f32", x, recv=np.array(recv, np.int32), seed=P)
    for r in range(P):
        assert (y[r, 0, :recv[r]] == P * (P - 1) / 2).all()


def test_multi_pointer_and_plan_shapes():
    steps, arena = get_plan("ring_chunked", 0, 4, 1000, 3)
    kinds = [s.kind for s in steps]
    assert kinds[0] == 8 and kinds[-1] == 9        # local reduce first, broadcast last
    assert arena == 2 * 256                         # two inboxes of max(256, ceil(n/2P))
    steps, arena = get_plan("local", 0, 1, 10, 1)
    assert steps == [] and arena == 0


def test_simulator_detects_protocol_violation():
    """The simulator must reject a schedule whose notifications are dropped."""
    import plan_sim
    orig = plan_sim.get_plan

    def broken(*a, **kw):
        steps, arena = orig(*a, **kw)
        return [s for s in steps if s.kind not in (plan_sim.KIND["NOTIFY"], plan_sim.KIND["WAIT_NOTIFY"])], arena

    plan_sim.get_plan = broken
    try:
        x = np.random.default_rng(0).standard_normal((3, 1, 5000)).astype(np.float32)
        with pytest.raises(ProtocolError):
            for seed in range(20):
                plan_sim.simulate("ring_chunked", "sum", "f32", x, seed=seed)
    finally:
        plan_sim.get_plan = orig


@pytest.mark.parametrize("P", [2, 3, 4, 7])
@pytest.mark.parametrize("n,seg", [(1, 0), (100, 128), (1000, 128), (5000, 256), (3, 4)])
def test_new_style_allreduce_closed_form(P, n, seg):
    """The new-style ring at many segment counts (gloo/test/allreduce_test.cc:
    307-378 exercises maxSegmentSize=128): every element j sums to
    j*P*P + P*(P-1)/2 and every output equals output 0."""
    x = np.array([[np.arange(n, dtype=np.float64) * P + r] * 2 for r in range(P)], dtype=np.float64)
    y = simulate("allreduce_new", "sum", "f64", x, seed=n + P, max_seg=seg)
    want = np.arange(n, dtype=np.float64) * P * P * 2 + 2 * P * (P - 1) / 2
    for r in range(P):
        assert (y[r, 0] == want).all() and (y[r, 1] == want).all()


def _ring_chunked_keys():
    return [k for k in _keys() if k.startswith("ring_chunked/") and int(k.split("/")[3][1:]) <= 8]


@pytest.mark.parametrize("case", _ring_chunked_keys())
def test_mesh_ring_chunked_matches_reference_golden(golden_sched, case):
    """RING_CHUNKED_MESH (plan.cc planRingChunkedMesh) reproduces the
    reference AllreduceRingChunked's bytes although the data moves in two
    all-to-all hops instead of around the ring."""
    op, dtype = case.split("/")[1:3]
    x, want = golden_sched[case + "/in"], golden_sched[case + "/out"]
    for seed in (0, 1, 2):
        y = simulate("ring_chunked_mesh", op, dtype, x, seed=seed)
        for r in range(y.shape[0]):
            for j in range(y.shape[1]):
                assert (y[r, j].view(np.uint8) == want.view(np.uint8)).all(), (seed, r, j)


@pytest.mark.parametrize("op", ["sum", "product", "max", "min"])
@pytest.mark.parametrize("dtype", ["f32", "f16", "bf16", "i32"])
@pytest.mark.parametrize("P,n", [(2, 1000), (3, 5000), (5, 999), (7, 4099), (8, 100003), (8, 300), (6, 1)])
def test_mesh_equals_ring_chunked_bitwise(op, dtype, P, n):
    """Mesh vs ring plan on random data incl. NaN / signed zeros (max/min are
    not commutative there, so operand order matters), over THREE back-to-back
    runs under random interleavings: identical bytes, and no inbox is
    overwritten before its fold has read it."""
    rng = np.random.default_rng(P * 1000 + n)
    if dtype == "i32":
        x = rng.integers(-2**31, 2**31 - 1, size=(P, 1, n), dtype=np.int64).astype(np.int32)
    else:
        f = rng.standard_normal((P, 1, n)).astype(np.float32)
        f[rng.random(f.shape) < 0.02] = np.nan
        f[rng.random(f.shape) < 0.02] = -0.0
        f[rng.random(f.shape) < 0.02] = 0.0
        if dtype == "f32":
            x = f
        elif dtype == "f16":
            x = f.astype(np.float16).view(np.uint16)
        else:
            x = (f.view(np.uint32) >> 16).astype(np.uint16)
    want = simulate("ring_chunked", op, dtype, x, seed=7, runs=3)
    for seed in (0, 1):
        got = simulate("ring_chunked_mesh", op, dtype, x, seed=seed, runs=3)
        assert (got.view(np.uint8) == want.view(np.uint8)).all(), seed


@pytest.mark.parametrize("P,k", [(3, 2), (4, 3)])
def test_mesh_multi_pointer(golden_sched, P, k):
    """Several local pointers: local fold, mesh exchange, local broadcast."""
    rng = np.random.default_rng(P + k)
    x = rng.standard_normal((P, k, 2049)).astype(np.float32)
    want = simulate("ring_chunked", "sum", "f32", x, seed=0)
    got = simulate("ring_chunked_mesh", "sum", "f32", x, seed=1, runs=1)
    assert (got.view(np.uint8) == want.view(np.uint8)).all()


def test_mesh_rejects_more_than_8_ranks():
    with pytest.raises(RuntimeError):
        get_plan("ring_chunked_mesh", 0, 9, 1000)


def _mesh_golden_keys():
    out = []
    for k in _keys():
        algo, P = k.split("/")[0], int(k.split("/")[3][1:])
        if algo in ("ring_chunked", "halving_doubling", "reduce_scatter") and 2 <= P <= 8:
            out.append(k)
    return out


@pytest.mark.parametrize("case", _mesh_golden_keys())
def test_derived_mesh_plan_matches_reference_golden(golden_sched, case):
    """algo | GLOO_HIP_ALGO_MESH (gloo_amd/csrc/mesh.cc): the plan derived by
    running the reference schedule symbolically — raw pieces straight to the
    rank that finishes them, the same expression tree evaluated there —
    reproduces the reference's bytes for ring-chunked, halving-doubling
    (balanced-tree fold for power-of-two P, pairwise for binary blocks) and
    reduce-scatter."""
    algo, op, dtype = case.split("/")[:3]
    x, want = golden_sched[case + "/in"], golden_sched[case + "/out"]
    for seed in (0, 1):
        if algo == "reduce_scatter":
            recv = golden_sched[case + "/recv"]
            y = simulate("mesh_" + algo, op, dtype, x[:, None, :], recv=recv, seed=seed)
            got = np.concatenate([y[r, 0, :recv[r]] for r in range(len(recv))])
            assert (got.view(np.uint8) == want.view(np.uint8)).all(), seed
        else:
            y = simulate("mesh_" + algo, op, dtype, x, seed=seed)
            for r in range(y.shape[0]):
                for j in range(y.shape[1]):
                    assert (y[r, j].view(np.uint8) == want.view(np.uint8)).all(), (seed, r, j)


def _random(dtype, shape, seed):
    rng = np.random.default_rng(seed)
    if dtype == "i32":
        return rng.integers(-2**31, 2**31 - 1, size=shape, dtype=np.int64).astype(np.int32)
    f = rng.standard_normal(shape).astype(np.float32)
    f[rng.random(shape) < 0.02] = np.nan
    f[rng.random(shape) < 0.02] = -0.0
    f[rng.random(shape) < 0.02] = 0.0
    if dtype == "f32":
        return f
    if dtype == "f16":
        return f.astype(np.float16).view(np.uint16)
    return (f.view(np.uint32) >> 16).astype(np.uint16)


@pytest.mark.parametrize("op", ["sum", "product", "max", "min"])
@pytest.mark.parametrize("dtype", ["f32", "bf16", "i32"])
@pytest.mark.parametrize("P,n", [(2, 1000), (3, 999), (4, 4099), (5, 1000), (6, 777), (7, 3001), (8, 100003),
                                 (8, 5)])
def test_mesh_hd_equals_hd_bitwise(op, dtype, P, n):
    """Derived mesh halving-doubling vs the reference schedule on random data
    with NaN / signed zeros, three back-to-back runs, random interleavings."""
    x = _random(dtype, (P, 1, n), P * 7 + n)
    want = simulate("halving_doubling", op, dtype, x, seed=3, runs=3)
    got = simulate("mesh_halving_doubling", op, dtype, x, seed=P, runs=3)
    assert (got.view(np.uint8) == want.view(np.uint8)).all()


@pytest.mark.parametrize("op", ["sum", "max"])
@pytest.mark.parametrize("dtype", ["f16", "bf16", "f32"])
@pytest.mark.parametrize("P,n", [(2, 100), (3, 1001), (5, 4099), (8, 4096), (8, 9)])
def test_mesh_reduce_scatter_bitwise_and_credits(op, dtype, P, n):
    """Derived mesh reduce-scatter: run 1 equals the reference's outputs;
    three back-to-back runs (no return hop, so inbox reuse rests on the
    previous-run credits) equal three single runs chained by hand."""
    x = _random(dtype, (P, 1, n), P * 11 + n)
    base = n // P
    recv = np.array([base + (1 if r < n % P else 0) for r in range(P)], dtype=np.int32)
    ref = simulate("reduce_scatter", op, dtype, x, recv=recv, seed=2)
    once = simulate("mesh_reduce_scatter", op, dtype, x, recv=recv, seed=1)
    for r in range(P):
        assert (once[r, 0, :recv[r]].view(np.uint8) == ref[r, 0, :recv[r]].view(np.uint8)).all(), r
    chained = x
    for _ in range(3):
        chained = simulate("mesh_reduce_scatter", op, dtype, chained, recv=recv, seed=5)
    for seed in (0, 1, 2):
        got = simulate("mesh_reduce_scatter", op, dtype, x, recv=recv, seed=seed, runs=3)
        assert (got.view(np.uint8) == chained.view(np.uint8)).all(), seed


def test_mesh_ring_has_no_mesh_form():
    """AllreduceRing's ranks finish with different association orders, so no
    single owner tree exists; the derivation refuses instead of guessing."""
    with pytest.raises(RuntimeError):
        get_plan("mesh_ring", 0, 4, 1000)
