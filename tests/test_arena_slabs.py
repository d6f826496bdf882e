"""CPU: the split of cross-process inbox arenas into IPC slabs
(executor.cc arenaSegments, exported as gloo_hip_arena_slabs).

HIP IPC imports of 2 GiB and more hang on ROCm 7 / MI355X
(profiles/round3/r3t_*, r3u_*), so an arena above 1.75 GiB is several pool
slabs, none above 1.75 GiB (the largest size class below 2^31).  The layout
is only sound if no kernel ever sees a slab boundary: every arena range a
rank's own steps read or write, and every message a peer writes into it,
must lie inside one slab.  Checked here over the real plans of every
schedule at BASELINE's largest sizes and beyond, for every rank."""
import ctypes

import numpy as np
import pytest

import plan_sim as ps

SEG_MAX = 7 << 28
GRANULE = 2 << 20
KIND = {"DECL_RECV": 0, "SEND": 1, "REDUCE": 3}
SRC_ARENA, DST_ARENA = 1, 2


def slabs(algo, rank, P, count, recv=None, es=4):
    L = ps.plan_lib()
    L.gloo_hip_arena_slabs.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t,
                                       ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_uint64),
                                       ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
    rp = None
    if recv is not None:
        recv = np.ascontiguousarray(recv, dtype=np.int32)
        rp = recv.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
    out = (ctypes.c_uint64 * 64)()
    n = ctypes.c_size_t()
    rc = L.gloo_hip_arena_slabs(ps.ALGO[algo], rank, P, count, 0, 1, es, 0, rp, out, 32, ctypes.byref(n))
    if rc:
        return None
    return [(out[2 * k], out[2 * k + 1]) for k in range(n.value)]


def arena_ranges(steps, es=4):
    for s in steps:
        if s.kind == KIND["DECL_RECV"]:
            yield s.dst_off * es, (s.dst_off + s.length) * es
        elif s.kind == KIND["REDUCE"]:
            yield s.src_off * es, (s.src_off + s.length) * es
        else:
            if s.flags & SRC_ARENA:
                yield s.src_off * es, (s.src_off + s.length) * es
            if s.flags & DST_ARENA:
                yield s.dst_off * es, (s.dst_off + s.length) * es


def inside_one(segs, a, b):
    return a == b or any(s <= a and b <= e for s, e in segs)


CASES = [("mesh_halving_doubling", P, n) for P in (2, 3, 4, 8) for n in (1 << 29, 510_000_000, 1 << 30)] + \
        [("ring_chunked_mesh", P, n) for P in (2, 4, 8) for n in (1 << 29, 1 << 30)] + \
        [("halving_doubling", P, n) for P in (2, 3, 8) for n in (1 << 29, 1 << 30)] + \
        [("ring_chunked", P, 1 << 30) for P in (2, 8)] + \
        [("mesh_reduce_scatter", P, n) for P in (2, 8) for n in (1 << 29, 1 << 30)]


@pytest.mark.parametrize("algo,P,count", CASES)
def test_every_range_and_message_inside_one_slab(algo, P, count):
    recv = None
    if "reduce_scatter" in algo:
        recv = [count // P + (1 if r < count % P else 0) for r in range(P)]
    plans = [ps.get_plan(algo, r, P, count, recv=recv) for r in range(P)]
    for r in range(P):
        steps, arena = plans[r]
        bytes_ = (max(256, arena * 4) + GRANULE - 1) // GRANULE * GRANULE
        segs = slabs(algo, r, P, count, recv)
        if bytes_ <= SEG_MAX:
            assert segs == [], (r, segs)
            continue
        if segs is None:
            # refused: only when one inbox region alone exceeds a slab
            biggest = max(b - a for a, b in arena_ranges(steps))
            assert biggest > SEG_MAX, (algo, P, count, r)
            continue
        assert 1 <= len(segs) <= 16
        for (s0, e0), (s1, e1) in zip(segs, segs[1:]):
            assert e0 <= s1
        for s, e in segs:
            assert e - s + s % 256 <= SEG_MAX and e <= arena * 4
        for a, b in arena_ranges(steps):
            assert inside_one(segs, a, b), (r, a, b, segs)
        # every peer's message lands inside one of this rank's slabs
        region = {(s.peer, s.slot): s.dst_off for s in steps if s.kind == KIND["DECL_RECV"]}
        for q in range(P):
            if q == r:
                continue
            for s in plans[q][0]:
                if s.kind == KIND["SEND"] and s.peer == r:
                    a = (region[(q, s.slot)] + s.dst_off) * 4
                    assert inside_one(segs, a, a + s.length * 4), (q, "->", r, a, segs)


def test_two_gib_mesh_arena_is_two_one_gib_slabs():
    """VERDICT r3 #2's case: HD at P = 2 with 2^29 fp32 per rank."""
    assert slabs("mesh_halving_doubling", 0, 2, 1 << 29) == [(0, 1 << 30), (1 << 30, 2 << 30)]
    # between 1.75 and 2 GiB: split too, never one 2 GiB size class
    assert len(slabs("mesh_halving_doubling", 0, 2, 510_000_000)) == 2
    # at or below 1.75 GiB: one block, as before
    assert slabs("mesh_halving_doubling", 0, 2, 7 << 26) == []


def test_unaligned_atom_at_the_limit_is_refused():
    """an atom's slab is its length plus its start's residue mod
    256 B.  A region of 1.75 GiB - 4 B starting 252 B past a 256 B boundary
    would need 1.75 GiB + 248 B, the 2 GiB size class (the hanging import):
    refused.  The same region 256-aligned (rank 0's first one) fits."""
    L = SEG_MAX // 4 - 1
    recv = [L, L, L]
    steps, _ = ps.get_plan("mesh_reduce_scatter", 0, 3, 3 * L, recv=recv)
    atoms = sorted(set(arena_ranges(steps)))
    assert atoms[1][0] % 256 == 252 and atoms[1][1] - atoms[1][0] <= SEG_MAX
    assert atoms[1][1] - atoms[1][0] + atoms[1][0] % 256 > SEG_MAX
    assert slabs("mesh_reduce_scatter", 0, 3, 3 * L, recv) is None
    # one element shorter per rank still leaves an unaligned start, but its slab fits
    L2 = SEG_MAX // 4 - 64
    segs = slabs("mesh_reduce_scatter", 0, 3, 3 * L2, [L2] * 3)
    assert segs and all(e - s + s % 256 <= SEG_MAX for s, e in segs)
