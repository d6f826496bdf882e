"""CPU: the one-launch interpreter's batching rule (signal.h kInterpDefer,
executor_run.cc markInterpBatches, exported as gloo_hip_interp_batches).

The interpreter kernel (reduce.hip plan_interp_kernel) drains memory and
passes a workgroup barrier only at the LAST step of a batch, so every pair of
data steps inside one batch must be independent — not just neighbours.  A
SIGNAL touches no bytes, so a neighbour-only check let the halving-doubling
reduce-scatter's REDUCE -> NOTIFY -> SEND-from-inside-the-reduced-range
(gloo/allreduce_halving_doubling.h:262-296, plan.cc planHalvingDoubling)
send bytes other waves had not stored yet.

The interpreter lists are rebuilt here the way buildInterp() emits them,
over fake addresses (only compared, never dereferenced), from the real
plans of every schedule, and every batch is checked pairwise."""
import ctypes

import pytest

import plan_sim as ps

K = ps.KIND
COPY, SEND, SIGNAL, WAIT, FOLD = 0, 1, 2, 3, 4
MAX_SRCS = 8


class Desc(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("nsrc", ctypes.c_int32), ("dst", ctypes.c_uint64),
                ("src", ctypes.c_uint64 * MAX_SRCS), ("bytes", ctypes.c_uint64)]


def batches(descs):
    L = ps.plan_lib()
    L.gloo_hip_interp_batches.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    arr = (Desc * max(1, len(descs)))()
    for i, (kind, dst, srcs, nbytes) in enumerate(descs):
        arr[i].kind, arr[i].nsrc, arr[i].dst, arr[i].bytes = kind, len(srcs), dst, nbytes
        for j, s in enumerate(srcs):
            arr[i].src[j] = s
    out = (ctypes.c_int * max(1, len(descs)))()
    assert L.gloo_hip_interp_batches(ctypes.cast(arr, ctypes.c_void_p), len(descs), out) == 0
    return [out[i] for i in range(len(descs))]


USER, INPUT, ARENA, PEER = 1 << 40, 2 << 40, 3 << 40, 4 << 40


def interp_list(steps, es=4):
    """buildInterp()'s list for one pointer, addresses symbolic."""
    decl = {}
    out, fold_srcs = [], []
    for s in steps:
        n = s.length * es
        if s.kind == K["DECL_RECV"]:
            decl[(s.peer, s.slot)] = s.dst_off
        elif s.kind == K["SEND"]:
            src = (ARENA if s.flags & ps.SRC_ARENA else INPUT if s.flags & ps.FROM_INPUTS else USER) + s.src_off * es
            dst = PEER + (s.peer << 36) + (s.slot << 32) + s.dst_off * es
            out.append((SEND, dst, [src], n))
        elif s.kind == K["NOTIFY"]:
            out.append((SIGNAL, 0, [], 0))
        elif s.kind in (K["WAIT_RECV"], K["WAIT_NOTIFY"]):
            out.append((WAIT, 0, [], 0))
        elif s.kind == K["REDUCE"]:
            a = (INPUT if s.flags & ps.FROM_INPUTS else USER) + s.dst_off * es
            out.append((FOLD, USER + s.dst_off * es, [a, ARENA + s.src_off * es], n))
        elif s.kind == K["COPY"]:
            dst = (ARENA if s.flags & ps.DST_ARENA else USER) + s.dst_off * es
            src = (ARENA if s.flags & ps.SRC_ARENA else USER) + s.src_off * es
            if dst != src and n:
                out.append((COPY, dst, [src], n))
        elif s.kind == K["FOLD_SRC"]:
            fold_srcs.append((ARENA if s.flags & ps.SRC_ARENA else INPUT if s.flags & ps.FROM_INPUTS else USER)
                             + s.src_off * es)
        elif s.kind == K["FOLD"]:
            dst = (ARENA if s.flags & ps.DST_ARENA else USER) + s.dst_off * es
            out.append((FOLD, dst, fold_srcs, n))
            fold_srcs = []
        elif s.kind == K["LOCAL_REDUCE"] and s.flags & ps.FROM_INPUTS:
            out.append((COPY, USER + s.dst_off * es, [INPUT + s.dst_off * es], n))
    return out


def ranges(d):
    kind, dst, srcs, n = d
    if kind in (SIGNAL, WAIT):
        return [], []
    return [(s, s + n) for s in srcs], [(dst, dst + n)]


def meet(x, y):
    return any(a < d and c < b for a, b in x for c, d in y)


def check_batches(lst, defer):
    """Every batch is one class and its data steps are pairwise independent."""
    start = 0
    for i in range(len(lst)):
        if defer[i]:
            assert i + 1 < len(lst)
            continue
        batch = lst[start:i + 1]
        waits = [d[0] == WAIT for d in batch]
        assert all(waits) or not any(waits), batch
        for a in range(len(batch)):
            ra, wa = ranges(batch[a])
            for b in range(a + 1, len(batch)):
                rb, wb = ranges(batch[b])
                assert not (meet(wa, rb) or meet(wa, wb) or meet(ra, wb)), (start + a, start + b)
        start = i + 1


def test_signal_does_not_bridge_a_dependency():
    """REDUCE user[0,400) ; NOTIFY ; SEND from user[0,200): the SEND must not
    share the REDUCE's batch (it reads what the fold stores)."""
    lst = [(FOLD, USER, [USER, ARENA], 400), (SIGNAL, 0, [], 0), (SEND, PEER, [USER], 200)]
    d = batches(lst)
    assert d[1] == 0, d  # the drain comes after the NOTIFY, before the SEND
    check_batches(lst, d)


def test_independent_runs_still_batch():
    lst = [(SEND, PEER, [USER], 64), (SIGNAL, 0, [], 0), (SEND, PEER + 64, [USER + 64], 64),
           (WAIT, 0, [], 0), (WAIT, 0, [], 0), (COPY, USER + 1024, [ARENA], 64)]
    assert batches(lst) == [1, 1, 0, 1, 0, 0]


def test_empty_and_single():
    assert batches([]) == []
    assert batches([(SEND, PEER, [USER], 64)]) == [0]


CASES = [(a, P, n) for a in ("halving_doubling", "reduce_scatter", "ring_chunked", "ring_chunked_pipe", "ring",
                             "mesh_halving_doubling", "mesh_reduce_scatter", "ring_chunked_mesh", "allreduce_bcube",
                             "allreduce_new", "reduce")
         for P in (2, 3, 4, 8) for n in (1, 37, 1000, 4099)]


@pytest.mark.parametrize("algo,P,count", CASES)
def test_every_batch_of_every_plan_is_independent(algo, P, count):
    recv = None
    if "reduce_scatter" in algo:
        recv = [count // P + (1 if r < count % P else 0) for r in range(P)]
    if algo == "reduce":
        recv = [0] + [0] * (P - 1)
    nin = 1 if algo in ("allreduce_new", "allreduce_bcube", "reduce") else 0
    for r in range(P):
        try:
            steps, _ = ps.get_plan(algo, r, P, count, recv=recv, nin=nin)
        except RuntimeError:
            pytest.skip("no plan for this shape")
        lst = interp_list(steps)
        check_batches(lst, batches(lst))


def test_hd_reduce_scatter_shape_is_split():
    """The reported case on a real plan: some HD rank at P=4 has a REDUCE,
    NOTIFY, SEND whose source lies in the reduced range, and no batch
    holds both."""
    found = False
    for r in range(4):
        steps, _ = ps.get_plan("halving_doubling", r, 4, 4099)
        lst = interp_list(steps)
        d = batches(lst)
        for i in range(len(lst) - 2):
            a, b, c = lst[i:i + 3]
            if a[0] == FOLD and b[0] == SIGNAL and c[0] == SEND and meet(ranges(a)[1], ranges(c)[0]):
                found = True
                assert not (d[i] and d[i + 1]), (r, i)
        check_batches(lst, d)
    assert found
