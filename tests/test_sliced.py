"""The sliced plan interpreter's contract on CPU (signal.h, executor.cc
sliceable): every rank runs its whole plan once per slice, each (rank, slice)
on its own flags and never waiting for another slice.  The rule the executor
applies before choosing that form is restated in plan_sim.sliceable; here
every reference golden whose plans satisfy it is executed sliced by the
simulator — every (rank, slice) an independent process, interleaved at
random — and must still give the reference's bytes.  The GPU side checks the
executor picks the same slice count (test_collectives_gpu.py).
"""
import os

import numpy as np
import pytest

from plan_sim import simulate, slice_range, sliceable

ES = {"f16": 2, "bf16": 2, "f32": 4, "f64": 8, "i32": 4, "i8": 1, "u8": 1, "i64": 8, "u64": 8}


def _cases():
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "sched_golden.npz"))
    out = []
    for case in sorted({k.rsplit("/", 1)[0] for k in z.files}):
        algo, P = case.split("/")[0], int(case.split("/")[3][1:])
        if algo in ("ring_chunked", "halving_doubling", "reduce_scatter", "ring"):
            out.append((case, algo))
            if 2 <= P <= 8 and algo != "ring":
                out.append((case, "mesh_" + algo))
            if 2 <= P <= 8 and algo == "ring_chunked":
                out.append((case, "ring_chunked_mesh"))  # the executor's default ring-chunked plan
    return out


def _all_sliceable(algo, P, n, k, recv, es):
    return all(sliceable(algo, P, n, r, k=k, recv=recv, elem_size=es) for r in range(P))


def test_slice_range_partitions():
    for es in (1, 2, 4, 8):
        for length in (0, 1, 7, 100, 4099, 65536):
            for G in (1, 2, 3, 7, 32):
                parts = [slice_range(length, g, G, es) for g in range(G)]
                assert parts[0][0] == 0 and parts[-1][1] == length
                for (a, b), (c, d) in zip(parts, parts[1:]):
                    assert b == c and a <= b
                # every boundary but the end is 16-byte granular
                assert all((a * es) % 16 == 0 for a, _ in parts if a < length)


@pytest.mark.parametrize("case,algo", _cases())
def test_sliced_execution_matches_reference(golden_sched, case, algo):
    parts = case.split("/")
    op, dtype, P = parts[1], parts[2], int(parts[3][1:])
    es = ES[dtype]
    x = golden_sched[case + "/in"]
    want = golden_sched[case + "/out"]
    recv = golden_sched[case + "/recv"] if parts[0] == "reduce_scatter" else None
    inputs = x[:, None, :] if parts[0] == "reduce_scatter" else x
    n, k = inputs.shape[2], inputs.shape[1]
    if not _all_sliceable(algo, P, n, k, recv, es):
        pytest.skip("not sliceable: runs as one workgroup")
    for slices, seed in ((2, 0), (3, 1), (7, 2)):
        y = simulate(algo, op, dtype, inputs, recv=recv, seed=seed, slices=slices)
        if parts[0] == "reduce_scatter":
            got = np.concatenate([y[r, 0, :recv[r]] for r in range(P)])
            assert (got.view(np.uint8) == want.view(np.uint8)).all(), slices
        elif parts[0] == "ring":
            assert (y[:, 0].view(np.uint8) == want.view(np.uint8)).all(), slices
        else:
            for r in range(P):
                for j in range(k):
                    assert (y[r, j].view(np.uint8) == want.view(np.uint8)).all(), (slices, r, j)


@pytest.mark.parametrize("algo,P", [("mesh_halving_doubling", 2), ("mesh_halving_doubling", 4),
                                    ("mesh_halving_doubling", 8), ("mesh_halving_doubling", 5),
                                    ("ring_chunked_mesh", 8), ("mesh_reduce_scatter", 8)])
def test_default_routes_are_sliceable(algo, P):
    """The plans a multi-GPU run takes by default (the derived mesh plans)
    slice consistently."""
    n = 262144
    recv = None
    if "reduce_scatter" in algo:
        recv = np.array([n // P + (1 if r < n % P else 0) for r in range(P)], np.int32)
    assert _all_sliceable(algo, P, n, 1, recv, 4)


@pytest.mark.parametrize("algo", ["ring_chunked", "halving_doubling"])
def test_refused_plans_would_be_wrong_sliced(algo):
    """The reference routes of ring-chunked and halving-doubling at P = 3 are
    refused by the rule (a later step reads a range with other boundaries
    than the step that wrote it).  Run sliced anyway, the simulator produces
    other bytes or a protocol violation within a few interleavings, so the
    rule guards a real hazard."""
    P, n = 3, 1000
    assert not _all_sliceable(algo, P, n, 1, None, 4)
    x = np.random.default_rng(3).standard_normal((P, 1, n)).astype(np.float32)
    want = simulate(algo, "sum", "f32", x, seed=0)
    wrong = False
    for seed in range(4):
        try:
            y = simulate(algo, "sum", "f32", x, seed=seed, slices=7)
        except AssertionError:
            wrong = True
            break
        if not (y.view(np.uint8) == want.view(np.uint8)).all():
            wrong = True
            break
    assert wrong


def _new_style_cases():
    d = os.path.join(os.path.dirname(__file__), "golden")
    out = []
    z = np.load(os.path.join(d, "newstyle_golden.npz"))
    for case in sorted({k.rsplit("/", 1)[0] for k in z.files}):
        if 2 <= int(case.split("/")[3][1:]) <= 8:
            out.append(("new", case))
    z = np.load(os.path.join(d, "sched_golden.npz"))
    for case in sorted({k.rsplit("/", 1)[0] for k in z.files if k.startswith("allreduce_new/")}):
        if 2 <= int(case.split("/")[3][1:]) <= 8:
            out.append(("sched", case))
    return out


@pytest.fixture(scope="module")
def golden_new():
    return np.load(os.path.join(os.path.dirname(__file__), "golden", "newstyle_golden.npz"))


@pytest.mark.parametrize("src,case", _new_style_cases())
def test_sliced_new_style_matches_reference(golden_sched, golden_new, src, case):
    """The new-style collectives' mesh plans (gloo::allreduce RING / BCUBE,
    gloo::reduce) sliced: their whole-range local steps (reduceInputs /
    broadcastOutputs) are split at the boundaries the exchange uses, after
    which every (rank, slice) runs alone and the bytes are the reference's
    (the root's output for reduce)."""
    g = golden_new if src == "new" else golden_sched
    parts = case.split("/")
    kind, op, dtype, P, nin = parts[0], parts[1], parts[2], int(parts[3][1:]), int(parts[4][1:])
    algo = {"bcube": "mesh_allreduce_bcube", "allreduce_new": "mesh_allreduce_new", "reduce": "mesh_reduce"}[kind]
    seg = int(parts[7][1:])
    init = g[case + "/init"]
    ins = g[case + "/in"] if nin else None
    want = g[case + "/out"]
    root = int(parts[6][1:]) if kind == "reduce" else None
    recv = np.array([root], np.int32) if kind == "reduce" else None
    n, k = init.shape[2], init.shape[1]
    es = ES[dtype] if dtype in ES else init.dtype.itemsize
    if not all(sliceable(algo, P, n, r, k=k, nin=nin, recv=recv, elem_size=es, max_seg=seg) for r in range(P)):
        pytest.skip("not sliceable")
    for slices, seed in ((2, 0), (5, 1)):
        y = simulate(algo, op, dtype, init, recv=recv, seed=seed, ins=ins, max_seg=seg, slices=slices)
        if kind == "reduce":  # only the root's output is defined on the mesh route
            assert (y[root, 0].view(np.uint8) == want[root].view(np.uint8)).all(), slices
            continue
        for r in range(P):
            for j in range(k):
                assert (y[r, j].view(np.uint8) == want.view(np.uint8)).all(), (slices, r, j)


def test_many_segment_plans_are_not_proposed_for_slicing():
    """A sliced plan has no fallback route, so a rank proposes slicing only if
    its device step list fits (executor_modes.cc slicedInterpSteps).  The new-style
    gloo::reduce on the reference route at 256 MiB with 1 MiB segments, 4 ranks
    (the 4-rank bench rehearsal that failed before the bound existed), needs
    far more than the 512 entries; the small default test plans fit."""
    from plan_sim import INTERP_MAX_STEPS, sliced_interp_steps
    n = (256 << 20) // 4
    recv = np.array([0], np.int32)
    big = [sliced_interp_steps("reduce", 4, n, r, nin=1, recv=recv, max_seg=1 << 20) for r in range(4)]
    assert max(big) > INTERP_MAX_STEPS, big
    small = [sliced_interp_steps("reduce", 4, 4097, r, nin=1, recv=recv, max_seg=256 << 10) for r in range(4)]
    assert max(small) <= INTERP_MAX_STEPS, small
    ring = [sliced_interp_steps("mesh_allreduce_new", 4, 1001, r, nin=1, max_seg=128 << 10) for r in range(4)]
    assert 0 < max(ring) <= INTERP_MAX_STEPS, ring
