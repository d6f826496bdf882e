"""CPU: the pipelined ring route of AllreduceRingChunked (plan.cc
planRingChunkedPipe).

The reference's ring rounds (gloo/allreduce_ring_chunked.h:141-157) with
three inboxes per channel, each round's reduce and the send of its result in
one FOLD + SEND window (fused by the executor into one fold_send launch).
Checked on the plan simulator (tests/plan_sim.py: every rank a process,
random interleavings, a send into an unconsumed inbox or a deadlock is an
error): the reference's bytes at every golden, over three back-to-back runs
with no barrier, at P = 2 ... 32 (the reference's P grid), with NaN and
signed zeros; and every round of a run is a fusable window."""
import numpy as np
import pytest

import plan_sim as ps
from test_fold_forward_plan import _fusable_windows


def _keys(golden):
    return [k.rsplit("/", 1)[0] for k in golden.files if k.startswith("ring_chunked/") and k.endswith("/in")]


def test_goldens_bitwise(golden_sched):
    keys = _keys(golden_sched)
    assert len(keys) >= 10
    for case in keys:
        op, dtype = case.split("/")[1:3]
        x, want = golden_sched[case + "/in"], golden_sched[case + "/out"]
        for seed in (0, 1):
            y = ps.simulate("ring_chunked_pipe", op, dtype, x, seed=seed)
            for r in range(y.shape[0]):
                for j in range(y.shape[1]):
                    assert (y[r, j].view(np.uint8) == want.view(np.uint8)).all(), (case, seed, r, j)


@pytest.mark.parametrize("op", ["sum", "max", "min"])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("P,n", [(2, 1000), (3, 5000), (4, 10007), (5, 7), (8, 100003), (8, 300), (6, 1),
                                 (13, 4099), (32, 1000)])
def test_equals_reference_ring_three_runs(op, dtype, P, n):
    """Random data incl. NaN / +-0 (max/min are not commutative there), three
    back-to-back runs under random interleavings: the reference ring's bytes,
    no inbox overwritten before it was read, no deadlock (the third inbox:
    a send waits for the right's credit of an earlier round, never of its
    own)."""
    rng = np.random.default_rng(P * 1000 + n)
    f = rng.standard_normal((P, 1, n)).astype(np.float32)
    f[rng.random(f.shape) < 0.02] = np.nan
    f[rng.random(f.shape) < 0.02] = -0.0
    x = f if dtype == "f32" else (f.view(np.uint32) >> 16).astype(np.uint16)
    want = ps.simulate("ring_chunked", op, dtype, x, seed=7, runs=3)
    for seed in (0, 1):
        got = ps.simulate("ring_chunked_pipe", op, dtype, x, seed=seed, runs=3)
        assert (got.view(np.uint8) == want.view(np.uint8)).all(), seed


@pytest.mark.parametrize("P", [2, 3, 4, 8])
def test_every_round_fuses(P):
    """Each round with a non-empty chunk is a FOLD + SEND (+ credit) window:
    2P - 2 reduce rounds and 2P - 4 forwarding allgather rounds."""
    n = 1 << 16
    for r in range(P):
        steps = ps.get_plan("ring_chunked_pipe", r, P, n)[0]
        assert _fusable_windows(steps) == (2 * P - 2) + (2 * P - 4), r


def test_multi_pointer():
    rng = np.random.default_rng(3)
    x = rng.standard_normal((4, 3, 2049)).astype(np.float32)
    want = ps.simulate("ring_chunked", "sum", "f32", x, seed=0)
    got = ps.simulate("ring_chunked_pipe", "sum", "f32", x, seed=1, runs=2)
    want2 = ps.simulate("ring_chunked", "sum", "f32", x, seed=0, runs=2)
    assert (got.view(np.uint8) == want2.view(np.uint8)).all()
    assert want.shape == got.shape
