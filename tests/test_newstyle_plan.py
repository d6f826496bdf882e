"""CPU: the new-style function collectives beyond the RING allreduce —
gloo::allreduce(opts) with BCUBE (gloo/allreduce.cc:397-669) and
gloo::reduce(opts) (gloo/reduce.cc:21-247) — restated as plans
(gloo_amd/csrc/plan.cc) and executed by the all-rank CPU simulator.

tests/golden/newstyle_golden.npz holds the reference's own outputs for these
two functions (oracle/gen_golden.py, ranks as threads over the reference's TCP
transport).  The closed-form grids mirror gloo/test/allreduce_test.cc:307-378
(AllreduceNewBcube) and gloo/test/reduce_test.cc:24-89 (ReduceTest): uint64
fixture src[j] = j*stride + id, maxSegmentSize 128, in place and not.
"""
import os

import numpy as np
import pytest

from plan_sim import KIND, SRC_ARENA, get_plan, simulate

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "newstyle_golden.npz")


def _keys(prefix):
    z = np.load(GOLDEN)
    return sorted({k.rsplit("/", 1)[0] for k in z.files if k.startswith(prefix)})


@pytest.fixture(scope="module")
def golden_new():
    return np.load(GOLDEN)


def same_bytes(a, b):
    return a.shape == b.shape and (a.view(np.uint8) == b.view(np.uint8)).all()


@pytest.mark.parametrize("case", _keys("bcube/"))
def test_bcube_matches_reference_golden(golden_new, case):
    parts = case.split("/")
    op, dtype = parts[1], parts[2]
    nin, seg = int(parts[4][1:]), int(parts[7][1:])
    init = golden_new[case + "/init"]
    ins = golden_new[case + "/in"] if nin else None
    want = golden_new[case + "/out"]
    for seed in (0, 1, 2):
        y = simulate("allreduce_bcube", op, dtype, init, seed=seed, ins=ins, max_seg=seg)
        for r in range(y.shape[0]):
            for j in range(y.shape[1]):
                assert same_bytes(y[r, j], want), (seed, r, j)


@pytest.mark.parametrize("case", _keys("reduce/"))
def test_reduce_matches_reference_golden(golden_new, case):
    """Every rank's whole output buffer (not only the root's) equals the
    reference's: the ring part writes partial sums into every rank's output,
    and the plan reproduces those writes too."""
    parts = case.split("/")
    op, dtype = parts[1], parts[2]
    nin, root, seg = int(parts[4][1:]), int(parts[6][1:]), int(parts[7][1:])
    init = golden_new[case + "/init"]
    ins = golden_new[case + "/in"] if nin else None
    want = golden_new[case + "/out"]
    for seed in (0, 1, 2):
        y = simulate("reduce", op, dtype, init, recv=np.array([root], np.int32), seed=seed, ins=ins,
                     max_seg=seg)
        assert same_bytes(y[:, 0], want), seed


def _fixture(P, k, n):
    """gloo/test/base_test.h:184-236 Fixture<uint64_t>::assignValues:
    src[i][j] = j * stride + (rank * k + i), stride = P * k."""
    stride = P * k
    return np.array([[np.arange(n, dtype=np.uint64) * stride + (r * k + i) for i in range(k)]
                     for r in range(P)], dtype=np.uint64)


@pytest.mark.parametrize("P", [1, 2, 3, 4, 6, 7, 8, 12])
@pytest.mark.parametrize("k", [1, 2, 3])
@pytest.mark.parametrize("n", [0, 1, 10, 100, 1000])
@pytest.mark.parametrize("in_place", [True, False])
def test_bcube_closed_form_grid(P, k, n, in_place):
    """AllreduceNewBcube grid (gloo/test/allreduce_test.cc:369-378) widened to
    P in {3, 6, 8, 12} (factorisations 3, 2*3, 2*2*2, 2*2*3)."""
    x = _fixture(P, k, n)
    if in_place:
        y = simulate("allreduce_bcube", "sum", "u64", x, seed=P + n, max_seg=128)
    else:
        y = simulate("allreduce_bcube", "sum", "u64", np.zeros_like(x), seed=P + n, ins=x, max_seg=128)
    stride = P * k
    want = np.arange(n, dtype=np.uint64) * stride * stride + stride * (stride - 1) // 2
    for r in range(P):
        for j in range(k):
            assert (y[r, j] == want).all(), (r, j)


@pytest.mark.parametrize("P", [1, 2, 3, 4, 7])
@pytest.mark.parametrize("n", [0, 1, 10, 100, 1000, 10000])
@pytest.mark.parametrize("in_place", [True, False])
def test_reduce_closed_form_grid(P, n, in_place):
    """ReduceTest grid (gloo/test/reduce_test.cc:82-89): every rank takes its
    turn as root; the root's output is j*P*P + P*(P-1)/2."""
    x = _fixture(P, 1, n)
    want = np.arange(n, dtype=np.uint64) * P * P + P * (P - 1) // 2
    for root in range(P):
        if in_place:
            y = simulate("reduce", "sum", "u64", x, recv=np.array([root], np.int32), seed=root, max_seg=128)
        else:
            y = simulate("reduce", "sum", "u64", np.zeros_like(x), recv=np.array([root], np.int32),
                         seed=root, ins=x, max_seg=128)
        assert (y[root, 0] == want).all(), root


@pytest.mark.parametrize("P,n", [(2, 1000), (4, 4099), (7, 333), (8, 100003)])
def test_reduce_repeated_runs(P, n):
    """Three back-to-back runs with no barrier between them (the credits must
    keep every inbox and the root's gather region safe): in place, run r
    reduces run r-1's outputs, so three single runs chained by hand agree."""
    rng = np.random.default_rng(P + n)
    x = rng.integers(0, 1 << 20, size=(P, 1, n), dtype=np.uint64)
    root = np.array([P - 1], np.int32)
    chained = x
    for _ in range(3):
        chained = simulate("reduce", "sum", "u64", chained, recv=root, seed=9)
    for seed in (0, 1):
        got = simulate("reduce", "sum", "u64", x, recv=root, seed=seed, runs=3)
        assert (got == chained).all(), seed


@pytest.mark.parametrize("P,n", [(3, 1000), (6, 4099), (8, 100003), (12, 10), (12, 4099)])
def test_bcube_repeated_runs(P, n):
    rng = np.random.default_rng(P * 3 + n)
    x = rng.integers(0, 1 << 20, size=(P, 1, n), dtype=np.uint64)
    chained = x
    for _ in range(3):
        chained = simulate("allreduce_bcube", "sum", "u64", chained, seed=4)
    for seed in (0, 1):
        got = simulate("allreduce_bcube", "sum", "u64", x, seed=seed, runs=3)
        assert (got == chained).all(), seed


def test_bcube_p12_stale_inbox_read_explains_r05():
    """GPUTEST_r05's one red case (BCUBE P=12, ranks as threads on one GPU,
    coarse-grained inboxes): rank 3's element 0 (the first wrong result the
    test met) came back -1.9609444 instead of -3.8116968 in the second call,
    elements 1-9 right.  The plan is exact (test_bcube_repeated_runs above).
    The model of ONE stale read reproduces the wrong value bit for bit: rank
    8's phase-1 fold (step 13, its inbox [5, 10) from rank 9) reads the inbox
    as it stood at the end of the first run, when offset 5 held rank 10's
    phase-2 message (rank 8's region for rank 10 is [3, 6)).  Offsets 6-9
    still held rank 9's equal first-run data, so only element 0 is wrong.
    (With equal inputs in both calls, rank 10's SECOND-run message landing
    early gives the same value; the hardware path was not reproduced in
    isolation)  Inboxes that any peer writes are now
    fine-grained (executor.cc), which closes the cache-line path; the GPU
    side is test_newstyle_gpu.py::test_threads_inboxes_fine_grained."""
    z = np.load(os.path.join(ROOT, "tests", "golden", "newstyle_golden.npz"))
    case = "bcube/sum/f32/P12/i0/o1/n10/s0"
    init, want = z[case + "/init"], z[case + "/out"]
    end_of_run1 = []
    y1 = simulate("allreduce_bcube", "sum", "f32", init, seed=1, arenas_out=end_of_run1)
    assert (y1[:, 0] == want).all()
    steps, _ = get_plan("allreduce_bcube", 8, 12, 10)
    assert steps[13].kind == KIND["FOLD_SRC"] and steps[13].flags & SRC_ARENA and steps[13].src_off == 5
    y2 = simulate("allreduce_bcube", "sum", "f32", init, seed=2, arena_init=end_of_run1, stale={(8, 13)})
    assert [str(v) for v in y2[:, 0, 0]] == ["-1.9609444"] * 12
    assert (y2[:, 0, 1:] == want[1:]).all()


def test_reduce_rejects_bad_root():
    from plan_sim import get_plan
    with pytest.raises(RuntimeError):
        get_plan("reduce", 0, 4, 100, recv=np.array([4], np.int32), elem_size=8)


# ---- derived mesh plans of the new-style collectives (gloo_amd/csrc/mesh.cc) ----

def _random(dtype, shape, seed):
    rng = np.random.default_rng(seed)
    if dtype in ("i32", "u64"):
        return rng.integers(0, 1 << 30, size=shape, dtype=np.int64).astype(np.int32 if dtype == "i32" else np.uint64)
    f = rng.standard_normal(shape).astype(np.float32)
    f[rng.random(shape) < 0.02] = np.nan
    f[rng.random(shape) < 0.02] = -0.0
    f[rng.random(shape) < 0.02] = 0.0
    if dtype == "f32":
        return f
    if dtype == "f16":
        return f.astype(np.float16).view(np.uint16)
    return (f.view(np.uint32) >> 16).astype(np.uint16)


def _mesh_keys(prefix):
    return [k for k in _keys(prefix) if 2 <= int(k.split("/")[3][1:]) <= 8]


@pytest.mark.parametrize("case", _mesh_keys("bcube/"))
def test_mesh_bcube_matches_reference_golden(golden_new, case):
    """BCUBE's result with mesh data movement: the trees the reference builds
    (balanced for P = 2^k, pairwise otherwise) evaluated at their owners."""
    parts = case.split("/")
    op, dtype, nin = parts[1], parts[2], int(parts[4][1:])
    init = golden_new[case + "/init"]
    ins = golden_new[case + "/in"] if nin else None
    want = golden_new[case + "/out"]
    for seed in (0, 1):
        y = simulate("mesh_allreduce_bcube", op, dtype, init, seed=seed, ins=ins)
        for r in range(y.shape[0]):
            for j in range(y.shape[1]):
                assert same_bytes(y[r, j], want), (seed, r, j)


def _ring_new_keys():
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "sched_golden.npz"))
    keys = sorted({k.rsplit("/", 1)[0] for k in z.files if k.startswith("allreduce_new/")})
    return [k for k in keys if 2 <= int(k.split("/")[3][1:]) <= 8]


@pytest.mark.parametrize("case", _ring_new_keys())
def test_mesh_new_style_ring_matches_reference_golden(golden_sched, case):
    """gloo::allreduce RING (<= 1 MiB segments around the ring in the
    reference) as two all-to-all hops, same bytes."""
    parts = case.split("/")
    op, dtype, nin, seg = parts[1], parts[2], int(parts[4][1:]), int(parts[7][1:])
    init = golden_sched[case + "/init"]
    ins = golden_sched[case + "/in"] if nin else None
    want = golden_sched[case + "/out"]
    y = simulate("mesh_allreduce_new", op, dtype, init, seed=3, ins=ins, max_seg=seg)
    for r in range(y.shape[0]):
        for j in range(y.shape[1]):
            assert same_bytes(y[r, j], want), (r, j)


@pytest.mark.parametrize("case", _mesh_keys("reduce/"))
def test_mesh_reduce_root_matches_reference_golden(golden_new, case):
    """gloo::reduce with mesh data movement: the ROOT's output equals the
    reference's (the other ranks' outputs are scratch in both)."""
    parts = case.split("/")
    op, dtype = parts[1], parts[2]
    nin, root, seg = int(parts[4][1:]), int(parts[6][1:]), int(parts[7][1:])
    init = golden_new[case + "/init"]
    ins = golden_new[case + "/in"] if nin else None
    want = golden_new[case + "/out"]
    for seed in (0, 1):
        y = simulate("mesh_reduce", op, dtype, init, recv=np.array([root], np.int32), seed=seed, ins=ins,
                     max_seg=seg)
        assert same_bytes(y[root, 0], want[root]), seed


@pytest.mark.parametrize("op", ["sum", "product", "max", "min"])
@pytest.mark.parametrize("dtype", ["f32", "bf16", "i32"])
@pytest.mark.parametrize("P,n,seg", [(2, 1000, 0), (3, 999, 128), (5, 4099, 256), (6, 777, 64), (8, 20011, 0)])
def test_mesh_new_style_bitwise_random(op, dtype, P, n, seg):
    """Mesh vs reference route on random data with NaN / signed zeros, for
    RING and BCUBE allreduce (three chained in-place runs) and reduce to a
    rotating root (separate inputs, three runs)."""
    x = _random(dtype, (P, 1, n), P * 13 + n)
    for algo in ("allreduce_new", "allreduce_bcube"):
        want = simulate(algo, op, dtype, x, seed=1, runs=3, max_seg=seg)
        got = simulate("mesh_" + algo, op, dtype, x, seed=P, runs=3, max_seg=seg)
        assert same_bytes(got, want), algo
    root = np.array([n % P], np.int32)
    init = _random(dtype, (P, 1, n), n)
    want = simulate("reduce", op, dtype, init, recv=root, seed=2, ins=x, max_seg=seg)
    got = simulate("mesh_reduce", op, dtype, init, recv=root, seed=P, ins=x, runs=3, max_seg=seg)
    assert same_bytes(got[root[0], 0], want[root[0], 0])
