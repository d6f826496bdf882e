"""CPU: which plan shapes the executor may fuse into fold + forward launches
(executor_run.cc enqueue; reduce.hip fold_send_kernel), checked on the plan
simulator (tests/plan_sim.py) against the reference's goldens.

The executor fuses a FOLD with the SENDs of its result that follow it
directly: those sends already waited for everything the fold waited for, so
storing the result into the peers' inboxes during the fold changes no
ordering.  The reference routes never have that shape: their REDUCE is
followed by NOTIFY (the inbox credit to the left) and WAIT_NOTIFY (the credit
from the right) before the SEND.  Fusing there means waiting for the right
credit before the reduce; the simulator shows that ordering deadlocks
(single- and double-buffered credit chains wrap around the ring), which is
why the executor leaves the reference routes unfused."""
import numpy as np
import pytest

import plan_sim as ps


def _fusable_windows(steps):
    """FOLD into the user buffer followed only by SENDs of exactly its range
    (the executor's rule; every SEND of the run must qualify)."""
    n = 0
    for i, s in enumerate(steps):
        if s.kind != ps.KIND["FOLD"] or s.flags & ps.DST_ARENA or s.length == 0:
            continue
        j = i + 1
        while (j < len(steps) and steps[j].kind == ps.KIND["SEND"]
               and not steps[j].flags & (ps.SRC_ARENA | ps.FROM_INPUTS)
               and steps[j].src_off == s.dst_off and steps[j].length == s.length):
            j += 1
        if j > i + 1 and (j == len(steps) or steps[j].kind != ps.KIND["SEND"]):
            n += 1
    return n


@pytest.mark.parametrize("algo,P", [("mesh_halving_doubling", 2), ("mesh_halving_doubling", 4),
                                    ("mesh_halving_doubling", 8), ("ring_chunked_mesh", 3),
                                    ("ring_chunked_mesh", 8), ("mesh_allreduce_new", 4)])
def test_mesh_owners_fold_then_forward(algo, P):
    """Every rank of a power-of-two mesh allreduce (and every ring-chunked
    mesh owner) ends its job with a fusable FOLD + SENDs window."""
    n = 1 << 16
    per_rank = [_fusable_windows(ps.get_plan(algo, r, P, n)[0]) for r in range(P)]
    assert all(w >= 1 for w in per_rank), per_rank


@pytest.mark.parametrize("algo", ["halving_doubling", "ring_chunked"])
def test_reference_routes_have_no_fusable_window(algo):
    for P in (2, 3, 5, 8):
        for r in range(P):
            assert _fusable_windows(ps.get_plan(algo, r, P, 10007)[0]) == 0


@pytest.mark.parametrize("case", ["halving_doubling/sum/f32/P2/k1/n1000", "ring_chunked/sum/f32/P2/k1/n1000",
                                  "ring_chunked/sum/f32/P8/k1/n10007", "ring_chunked/sum/f64/P4/k1/n4099"])
def test_reduce_forward_on_reference_routes_deadlocks(golden_sched, case):
    """Moving each WAIT_NOTIFY before its REDUCE (what a fused reduce + send
    would need) deadlocks these reference schedules."""
    algo, op, dtype = case.split("/")[:3]
    x = golden_sched[case + "/in"]
    steps = ps.get_plan(algo, 0, x.shape[0], x.shape[-1])[0]
    assert ps.reduce_forward_order(steps)[1] > 0
    with pytest.raises(ps.ProtocolError, match="deadlock"):
        ps.simulate(algo, op, dtype, x, seed=0, reduce_forward=True)


@pytest.mark.parametrize("case", ["ring_chunked/sum/f32/P8/k1/n1000", "ring_chunked/max/f32/P5/k1/n999"])
def test_reduce_forward_where_it_happens_to_complete(golden_sched, case):
    """Where the rewritten order completes, it still gives the reference's
    bytes (the fused launch reduces, then forwards the same values)."""
    algo, op, dtype = case.split("/")[:3]
    x = golden_sched[case + "/in"]
    want = golden_sched[case + "/out"]
    for seed in range(3):
        y = ps.simulate(algo, op, dtype, x, seed=seed, reduce_forward=True)
        for r in range(x.shape[0]):
            assert (y[r, 0].view(np.uint8) == want.view(np.uint8)).all()
