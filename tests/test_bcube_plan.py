"""CPU: AllreduceBcube (gloo/allreduce_bcube.h; GPU twin CudaAllreduceBcube,
gloo/cuda_allreduce_bcube.{h,cc}) restated as a plan (gloo_amd/csrc/plan.cc
planBcube) and executed by the all-rank CPU simulator.

tests/golden/bcube_golden.npz holds the reference's own outputs, every rank's
(oracle/gen_golden.py bcube: AllreduceBcube<T> on contexts of base 2, 3 and 4,
ranks as threads over the reference's TCP transport): the P = base^k grid of
gloo/test/allreduce_test.cc:271-299 with n in {1, 64, 1000}, larger counts,
several pointers, f64 / bf16 / f16 / i32, max / min / product, and two rank
counts that are not powers of the base (the reference's ranges as they fall
there, which do not add up to a full allreduce — pinned, not endorsed).
"""
import math
import os

import numpy as np
import pytest

from plan_sim import KIND, get_plan, simulate

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "bcube_golden.npz")


def _keys():
    z = np.load(GOLDEN)
    return sorted({k.rsplit("/", 1)[0] for k in z.files})


def _parse(case):
    _, op, dtype, P, b, k, n = case.split("/")
    return op, dtype, int(P[1:]), int(b[1:]), int(k[1:]), int(n[1:])


@pytest.fixture(scope="module")
def golden():
    return np.load(GOLDEN)


def same_bytes(a, b):
    return a.shape == b.shape and (a.view(np.uint8) == b.view(np.uint8)).all()


@pytest.mark.parametrize("case", _keys())
def test_bcube_matches_reference_golden(golden, case):
    """Every rank's output (all its pointers) equals the reference's byte for
    byte, under two random rank interleavings."""
    op, dtype, P, base, k, n = _parse(case)
    x = golden[case + "/in"]
    want = golden[case + "/out"]
    for seed in (0, 1):
        y = simulate("bcube", op, dtype, x.copy(), recv=np.array([base], np.int32), seed=seed)
        for r in range(P):
            for j in range(k):
                assert same_bytes(np.asarray(y[r][j]), want[r]), (seed, r, j)


@pytest.mark.parametrize("case", ["bcube/sum/f32/P8/b2/k1/n1000", "bcube/sum/f32/P9/b3/k1/n64",
                                  "bcube/sum/f32/P16/b4/k1/n1000", "bcube/sum/f32/P4/b2/k3/n1000",
                                  "bcube/sum/f32/P6/b2/k1/n1000"])
def test_bcube_repeated_runs(golden, case):
    """Three back-to-back runs with no barrier between them (repeated
    Algorithm::run() calls): no message lands on an unconsumed one (the
    simulator raises on that), and each run's result is the one-run result of
    the previous run's outputs."""
    op, dtype, P, base, k, n = _parse(case)
    x = golden[case + "/in"]
    base_arr = np.array([base], np.int32)
    y3 = simulate("bcube", op, dtype, x.copy(), recv=base_arr, seed=3, runs=3)
    y = x.copy()
    for _ in range(3):
        y = simulate("bcube", op, dtype, np.ascontiguousarray(y), recv=base_arr, seed=4)
    for r in range(P):
        for j in range(k):
            assert same_bytes(np.asarray(y3[r][j]), np.asarray(y[r][j])), (r, j)


@pytest.mark.parametrize("P,base", [(2, 2), (4, 2), (8, 2), (16, 2), (3, 3), (9, 3), (27, 3), (4, 4), (16, 4),
                                    (6, 2), (5, 3)])
def test_bcube_geometry(P, base):
    """Steps = ceil(float log2 P / float log2 base) (gloo/allreduce_bcube.h:528-532);
    each step pairs a rank with the ranks base^step apart in its group; a
    peer meets a rank in one step only; sends and receives balance."""
    steps = math.ceil(np.float32(np.float32(math.log2(P)) / np.float32(math.log2(base))))
    n = 1000
    plans = [get_plan("bcube", r, P, n, 1, np.array([base], np.int32))[0] for r in range(P)]
    for r, st in enumerate(plans):
        peers = [s.peer for s in st if s.kind == KIND["DECL_RECV"]]
        assert len(peers) == len(set(peers)), (r, peers)
        for q in peers:
            d = abs(q - r)
            assert any(d == i * base ** s for s in range(steps) for i in range(1, base)), (r, q)
        assert len(peers) <= steps * (base - 1)
    sends = {}
    for r, st in enumerate(plans):
        for s in st:
            if s.kind == KIND["SEND"]:
                sends[(r, s.peer)] = sends.get((r, s.peer), 0) + 1
    waits = {}
    for r, st in enumerate(plans):
        for s in st:
            if s.kind == KIND["WAIT_RECV"]:
                waits[(s.peer, r)] = waits.get((s.peer, r), 0) + 1
    assert sends == waits


def test_bcube_base_defaults_to_two():
    """No base (gloo_hip_plan without recv_elems) plans base 2, as
    CudaAllreduceBcube takes `context->base ? context->base : 2`
    (gloo/cuda_allreduce_bcube.cc:57); so does base 0."""
    for r in range(8):
        a = get_plan("bcube", r, 8, 1000, 1, None)
        b = get_plan("bcube", r, 8, 1000, 1, np.array([2], np.int32))
        c = get_plan("bcube", r, 8, 1000, 1, np.array([0], np.int32))
        key = lambda p: [(s.kind, s.peer, s.slot, s.flags, s.dst_off, s.src_off, s.length) for s in p[0]]  # noqa: E731
        assert key(a) == key(b) == key(c)


def test_bcube_zero_count_and_single_rank():
    """count 0: nothing (run() :348-351); one rank: the local reduce and
    broadcast only (:357-363)."""
    assert len(get_plan("bcube", 0, 4, 0, 1, np.array([2], np.int32))[0]) == 0
    st, arena = get_plan("bcube", 0, 1, 100, 3, np.array([2], np.int32))
    assert [s.kind for s in st] == [KIND["LOCAL_REDUCE"], KIND["LOCAL_BCAST"]] and arena == 0


def _mesh_plans(P, base, n, k=1):
    """Every rank's derived mesh plan (gloo_amd/csrc/mesh.cc), or None where
    the derivation refuses (ranks ending with different expression trees,
    partial reductions, mixed element indices): the executor then keeps the
    reference route (executor.cc, the constructor's fallback)."""
    try:
        return [get_plan("mesh_bcube", r, P, n, k, np.array([base], np.int32)) for r in range(P)]
    except RuntimeError:
        return None


@pytest.mark.parametrize("case", [c for c in _keys() if 2 <= _parse(c)[2] <= 8])
def test_mesh_bcube_matches_reference_golden(golden, case):
    """Where the mesh form exists (the executor's default for 2 <= P <= 8) it
    gives the reference's bytes on every rank; it exists for every P = base^k
    case with n >= 64, and not where the reference's ranks end differently
    (P not a power of the base)."""
    op, dtype, P, base, k, n = _parse(case)
    plans = _mesh_plans(P, base, n, k)
    power = base ** round(math.log(P, base)) == P
    if power and n >= 64:
        assert plans is not None, case
    if not power:
        assert plans is None, case
    if plans is None:
        return
    x = golden[case + "/in"]
    want = golden[case + "/out"]
    for seed in (0, 1):
        y = simulate("mesh_bcube", op, dtype, x.copy(), recv=np.array([base], np.int32), seed=seed)
        for r in range(P):
            for j in range(k):
                assert same_bytes(np.asarray(y[r][j]), want[r]), (seed, r, j)
