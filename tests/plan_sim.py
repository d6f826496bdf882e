"""CPU simulation of gloo_amd plans — TEST INFRASTRUCTURE.

Executes the per-rank step lists produced by gloo_hip_plan (the C++
restatement of the reference schedules) for ALL ranks at once over numpy
buffers, with the oracle restatement of gloo/math.h as the reduction.  Sends
are one-sided writes into the receiver's declared inbox region, exactly the
semantics of gloo::transport::Buffer::send (gloo/transport/buffer.h:26-34).
The scheduler interleaves ranks in a seeded random order, and flags any send
that would overwrite a message the receiver has not consumed yet (a broken
notification protocol) and any deadlock.
"""
import ctypes
import random

import numpy as np

import oracle

KIND = dict(DECL_RECV=0, SEND=1, WAIT_RECV=2, REDUCE=3, COPY=4, NOTIFY=5, WAIT_NOTIFY=6,
            WAIT_SEND=7, LOCAL_REDUCE=8, LOCAL_BCAST=9, FOLD_SRC=10, FOLD=11)
ALGO = dict(ring_chunked=0, halving_doubling=1, ring=2, local=3, reduce_scatter=4, allreduce_new=5,
            ring_chunked_mesh=6, allreduce_bcube=7, reduce=8, ring_chunked_pipe=9, bcube=10)
MESH = 0x100  # algo | MESH: the derived mesh plan (gloo_amd/csrc/mesh.cc)
ALGO.update({"mesh_" + k: v | MESH for k, v in list(ALGO.items()) if v < 5 or v in (5, 7, 8, 10)})
SRC_ARENA, DST_ARENA, FROM_INPUTS, FOLD_REVERSE, FOLD_TREE, PREV_RUN = 1, 2, 4, 8, 16, 32


class Step(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("peer", ctypes.c_int32), ("slot", ctypes.c_int32),
                ("flags", ctypes.c_int32), ("dst_off", ctypes.c_uint64), ("src_off", ctypes.c_uint64),
                ("length", ctypes.c_uint64)]


_plan_lib = None


def plan_lib():
    """The planners' C-ABI: the product library, or (GLOO_AMD_PLAN_LIB) a
    host-only build of plan.cc + mesh.cc, e.g. under AddressSanitizer."""
    global _plan_lib
    if _plan_lib is None:
        import os
        path = os.environ.get("GLOO_AMD_PLAN_LIB")
        if path:
            _plan_lib = ctypes.CDLL(path)
        else:
            import gloo_amd
            _plan_lib = gloo_amd.lib
    return _plan_lib


def get_plan(algo, rank, size, count, nptrs=1, recv=None, nin=0, elem_size=4, max_seg=0):
    L = plan_lib()
    n = ctypes.c_size_t()
    arena = ctypes.c_size_t()
    rp = None
    if recv is not None:
        recv = np.ascontiguousarray(recv, dtype=np.int32)
        rp = recv.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
    L.gloo_hip_plan_ex.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t,
                                   ctypes.POINTER(ctypes.c_int), ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
    args = (ALGO[algo], rank, size, count, nin, nptrs, elem_size, max_seg, rp)
    rc = L.gloo_hip_plan_ex(*args, None, 0, ctypes.byref(n), ctypes.byref(arena))
    if rc:
        raise RuntimeError(f"gloo_hip_plan failed {rc}")
    steps = (Step * max(1, n.value))()
    rc = L.gloo_hip_plan_ex(*args, ctypes.cast(steps, ctypes.c_void_p), n.value, ctypes.byref(n),
                            ctypes.byref(arena))
    if rc:
        raise RuntimeError(f"gloo_hip_plan failed {rc}")
    return [steps[i] for i in range(n.value)], arena.value


class ProtocolError(AssertionError):
    pass


def slice_range(length, g, slices, elem_size):
    """Slice g of a step of `length` elements in the sliced interpreter
    (gloo_amd/include/gloo_amd/signal.h): q = ceil(length / slices) rounded
    up to 16 bytes, [min(length, g q), min(length, g q + q))."""
    kv = max(1, 16 // elem_size)
    q = -(-(-(-length // slices)) // kv) * kv
    lo = min(length, g * q)
    return lo, min(length, lo + q)


def user_cuts(steps):
    """Boundaries the non-local steps use in the user buffers (executor.cc
    userCuts): the sliced form splits whole-range local steps there."""
    c = set()
    for t in steps:
        K = t.kind
        if K in (KIND["SEND"], KIND["FOLD_SRC"]) and not t.flags & SRC_ARENA:
            c |= {t.src_off, t.src_off + t.length}
        elif K == KIND["REDUCE"]:
            c |= {t.dst_off, t.dst_off + t.length}
        elif K == KIND["COPY"]:
            if not t.flags & SRC_ARENA:
                c |= {t.src_off, t.src_off + t.length}
            if not t.flags & DST_ARENA:
                c |= {t.dst_off, t.dst_off + t.length}
        elif K == KIND["FOLD"] and not t.flags & DST_ARENA:
            c |= {t.dst_off, t.dst_off + t.length}
    return sorted(c)


def cut_range(cuts, off, length):
    out, at = [], off
    for c in cuts:
        if at < c < off + length:
            out.append((at, c - at))
            at = c
    if off + length > at:
        out.append((at, off + length - at))
    return out


def sliceable(algo, P, n, rank, k=1, nin=0, recv=None, elem_size=4, max_seg=0):
    """Python statement of the executor's rule (gloo_amd/csrc/executor.cc
    sliceable): may `rank` run its plan sliced?  Every read overlapping an
    earlier write (peers' messages into the arena count as written first)
    must be exactly that range; every write overlapping an earlier access
    must be exactly that range."""
    steps, _ = get_plan(algo, rank, P, n, k, recv, nin=nin, elem_size=elem_size, max_seg=max_seg)
    decl = {(s.peer, s.slot): s.dst_off for s in steps if s.kind == KIND["DECL_RECV"]}
    cuts = user_cuts(steps)
    reads, writes = {}, {}

    def clash(a, b):
        return a[0] < b[0] + b[1] and b[0] < a[0] + a[1] and a != b

    def write(buf, off, ln):
        if not ln:
            return True
        if any(clash(x, (off, ln)) for x in reads.get(buf, []) + writes.get(buf, [])):
            return False
        writes.setdefault(buf, []).append((off, ln))
        return True

    def read(buf, off, ln):
        if not ln:
            return True
        if any(clash(x, (off, ln)) for x in writes.get(buf, [])):
            return False
        reads.setdefault(buf, []).append((off, ln))
        return True

    ARENA, IN = -1, 1 << 20
    for peer in range(P):
        if peer == rank:
            continue
        theirs, _ = get_plan(algo, peer, P, n, 1, recv, nin=0, elem_size=elem_size, max_seg=max_seg)
        for t in theirs:
            if t.kind == KIND["SEND"] and t.peer == rank:
                if (peer, t.slot) not in decl or not write(ARENA, decl[(peer, t.slot)] + t.dst_off, t.length):
                    return False

    def send_buf(t):
        return ARENA if t.flags & SRC_ARENA else IN if t.flags & FROM_INPUTS else 0

    for t in steps:
        K, L = t.kind, t.length
        if K in (KIND["SEND"], KIND["FOLD_SRC"]):
            ok = read(send_buf(t), t.src_off, L)
        elif K == KIND["REDUCE"]:
            ok = read(IN if t.flags & FROM_INPUTS else 0, t.dst_off, L) and read(ARENA, t.src_off, L) and \
                write(0, t.dst_off, L)
        elif K == KIND["COPY"]:
            ok = read(ARENA if t.flags & SRC_ARENA else 0, t.src_off, L) and \
                write(ARENA if t.flags & DST_ARENA else 0, t.dst_off, L)
        elif K == KIND["FOLD"]:
            ok = write(ARENA if t.flags & DST_ARENA else 0, t.dst_off, L)
        elif K == KIND["LOCAL_REDUCE"]:
            from_in = t.flags & FROM_INPUTS
            ok = all(all(read((IN if from_in else 0) + j, o, ln) for j in range(nin if from_in else k)) and
                     write(0, o, ln) for o, ln in cut_range(cuts, t.dst_off, L))
        elif K == KIND["LOCAL_BCAST"]:
            ok = all(read(0, o, ln) and all(write(j, o, ln) for j in range(1, k))
                     for o, ln in cut_range(cuts, t.dst_off, L))
        else:
            ok = True
        if not ok:
            return False
    return True


def reduce_forward_order(steps):
    """The executor's reduce + forward rewrite (executor_run.cc enqueue): a window
    REDUCE(range R) NOTIFY WAIT_NOTIFY SEND(R, unchanged) runs as
    WAIT_NOTIFY, then ONE launch that reduces R and stores the result into
    the peer's inbox as it goes (here: REDUCE then SEND), then NOTIFY.
    Returns (new step list, number of windows rewritten)."""
    out, i, hits = [], 0, 0
    while i < len(steps):
        s = steps[i]
        if (s.kind == KIND["REDUCE"] and not s.flags & FROM_INPUTS and s.length > 0 and i + 3 < len(steps)
                and steps[i + 1].kind == KIND["NOTIFY"] and steps[i + 2].kind == KIND["WAIT_NOTIFY"]
                and steps[i + 3].kind == KIND["SEND"] and not steps[i + 3].flags & (SRC_ARENA | FROM_INPUTS)
                and steps[i + 3].src_off == s.dst_off and steps[i + 3].length == s.length):
            out += [steps[i + 2], s, steps[i + 3], steps[i + 1]]
            hits += 1
            i += 4
            continue
        out.append(s)
        i += 1
    return out, hits


def simulate(algo, op, dtype, inputs, recv=None, seed=0, ins=None, max_seg=0, runs=1, slices=1,
             reduce_forward=False, arena_init=None, stale=(), arenas_out=None):
    """inputs: [P][k][n] array of the dtype's storage type (the outputs'
    initial contents); ins: optional [P][kin][n] separate inputs (new-style
    allreduce).  runs > 1 executes the plan back to back that many times
    (each run reduces the previous run's outputs), with no barrier between
    runs, as repeated Algorithm::run() calls do.  slices > 1 executes it as
    the sliced interpreter does: every (rank, slice) is its own process
    applying each step to its slice only, with its own channel counters,
    interleaved at random with all the others.  reduce_forward: every plan
    rewritten by reduce_forward_order first.  arena_init: each rank's arena
    contents at the start (default zeros); stale: {(rank, step index)} of
    FOLD_SRC steps whose arena operand is read as it stood at the start (a
    stale cache line of the inbox, the fault model of GPUTEST_r05);
    arenas_out: a list that receives the final arenas.  Returns the outputs."""
    P, k, n = inputs.shape
    nin = 0 if ins is None else ins.shape[1]
    es = inputs.dtype.itemsize
    plans = [get_plan(algo, r, P, n, k, recv, nin=nin, elem_size=es, max_seg=max_seg) for r in range(P)]
    if reduce_forward:
        plans = [(reduce_forward_order(steps)[0], a) for steps, a in plans]
    # previous-run credits: per channel, how many per run
    lag_per_run = {}
    for r, (steps, _) in enumerate(plans):
        for st in steps:
            if st.kind == KIND["WAIT_NOTIFY"] and st.flags & PREV_RUN:
                key = (st.peer, r, st.slot)
                lag_per_run[key] = lag_per_run.get(key, 0) + 1
    if runs > 1:
        plans = [([st for st in steps] + [st for _ in range(runs - 1) for st in steps
                                          if st.kind != KIND["DECL_RECV"]], a) for steps, a in plans]
    user = [[inputs[r, j].copy() for j in range(k)] for r in range(P)]
    arena = [np.zeros(max(1, a), dtype=inputs.dtype) for _, a in plans]
    if arena_init is not None:
        for r in range(P):
            arena[r][:] = arena_init[r]
    arena0 = [a.copy() for a in arena]
    regions = {}
    for r, (steps, _) in enumerate(plans):
        for s in steps:
            if s.kind == KIND["DECL_RECV"]:
                key = (s.peer, r, s.slot)
                if key in regions:
                    raise ProtocolError(f"region {key} declared twice")
                regions[key] = (s.dst_off, s.length)
    sent, consumed, lagged = {}, {}, {}
    procs = [(r, g) for r in range(P) for g in range(slices)]
    pending = {p: [] for p in procs}  # FOLD sources, read when the FOLD executes
    pc = {p: 0 for p in procs}
    rng = random.Random(seed)

    def space(r, is_arena):
        return arena[r] if is_arena else user[r][0]

    def runnable(p):
        r, g = p
        steps = plans[r][0]
        if pc[p] >= len(steps):
            return False
        s = steps[pc[p]]
        if s.kind == KIND["WAIT_NOTIFY"] and s.flags & PREV_RUN:
            # the i-th such wait is met by the previous run's credits
            key = (s.peer, r, s.slot, g)
            return sent.get(key, 0) >= lagged.get(key, 0) + 1 - lag_per_run[key[:3]]
        if s.kind in (KIND["WAIT_RECV"], KIND["WAIT_NOTIFY"]):
            key = (s.peer, r, s.slot, g)
            return sent.get(key, 0) > consumed.get(key, 0)
        return True

    cuts = [user_cuts(steps) for steps, _ in plans]

    def local_step(r, s, lo, hi):
        out0 = user[r][0]
        if s.kind == KIND["LOCAL_BCAST"]:
            for j in range(1, k):
                user[r][j][lo:hi] = out0[lo:hi]
        elif s.flags & FROM_INPUTS:
            if nin == 1:
                out0[lo:hi] = ins[r, 0, lo:hi]
            else:
                out0[lo:hi] = oracle.reduce3(op, dtype, ins[r, 0, lo:hi], ins[r, 1, lo:hi])
                for j in range(2, nin):
                    out0[lo:hi] = oracle.reduce3(op, dtype, out0[lo:hi], ins[r, j, lo:hi])
        else:
            for j in range(1, k):
                out0[lo:hi] = oracle.reduce3(op, dtype, out0[lo:hi], user[r][j][lo:hi])

    while True:
        ready = [p for p in procs if runnable(p)]
        if not ready:
            if all(pc[p] >= len(plans[p[0]][0]) for p in procs):
                break
            raise ProtocolError(f"deadlock at pcs {pc}")
        r, g = rng.choice(ready)
        s = plans[r][0][pc[(r, g)]]
        pc[(r, g)] += 1
        K = s.kind
        a0, a1 = slice_range(s.length, g, slices, es)  # this process's part of the step
        if K == KIND["DECL_RECV"] or K == KIND["WAIT_SEND"]:
            continue
        if K == KIND["WAIT_NOTIFY"] and s.flags & PREV_RUN:
            key = (s.peer, r, s.slot, g)
            lagged[key] = lagged.get(key, 0) + 1
            continue
        if K == KIND["SEND"]:
            key = (r, s.peer, s.slot, g)
            if key[:3] not in regions:
                raise ProtocolError(f"send to undeclared region {key}")
            if sent.get(key, 0) > consumed.get(key, 0):
                raise ProtocolError(f"send {key} overwrites an unconsumed message")
            roff, cap = regions[key[:3]]
            if s.length > cap:
                raise ProtocolError(f"send {key} of {s.length} exceeds region {cap}")
            src = ins[r, 0] if s.flags & FROM_INPUTS else space(r, s.flags & SRC_ARENA)
            arena[s.peer][roff + a0:roff + a1] = src[s.src_off + a0:s.src_off + a1]
            sent[key] = sent.get(key, 0) + 1
        elif K in (KIND["WAIT_RECV"], KIND["WAIT_NOTIFY"]):
            key = (s.peer, r, s.slot, g)
            consumed[key] = consumed.get(key, 0) + 1
        elif K == KIND["NOTIFY"]:
            key = (r, s.peer, s.slot, g)
            sent[key] = sent.get(key, 0) + 1
        elif K == KIND["REDUCE"]:
            dst = user[r][0]
            # FROM_INPUTS: out = in op inbox (gloo::reduce, gloo/reduce.cc:180-184)
            a = (ins[r, 0] if s.flags & FROM_INPUTS else dst)[s.dst_off + a0:s.dst_off + a1]
            b = arena[r][s.src_off + a0:s.src_off + a1]
            dst[s.dst_off + a0:s.dst_off + a1] = oracle.reduce3(op, dtype, a, b)
        elif K == KIND["COPY"]:
            src = space(r, s.flags & SRC_ARENA)
            dst = space(r, s.flags & DST_ARENA)
            dst[s.dst_off + a0:s.dst_off + a1] = src[s.src_off + a0:s.src_off + a1].copy()
        elif K in (KIND["LOCAL_REDUCE"], KIND["LOCAL_BCAST"]):
            # sliced: the executor first splits whole-range local steps at the
            # user-buffer boundaries the other steps use (executor_modes.cc userCuts)
            pieces = cut_range(cuts[r], s.dst_off, s.length) if slices > 1 else [(s.dst_off, s.length)]
            for o, ln in pieces:
                b0, b1 = slice_range(ln, g, slices, es)
                local_step(r, s, o + b0, o + b1)
        elif K == KIND["FOLD_SRC"]:
            pending[(r, g)].append((s.flags, s.src_off, (r, pc[(r, g)] - 1) in stale))
        elif K == KIND["FOLD"]:
            srcs = [(ins[r, 0] if f & FROM_INPUTS else arena0[r] if old and f & SRC_ARENA
                     else space(r, f & SRC_ARENA))[o + a0:o + a1].copy()
                    for f, o, old in pending[(r, g)]]
            pending[(r, g)] = []
            if s.flags & FOLD_TREE:
                while len(srcs) > 1:
                    srcs = [oracle.reduce3(op, dtype, srcs[2 * j], srcs[2 * j + 1]) for j in range(len(srcs) // 2)]
                acc = srcs[0]
            else:
                acc = srcs[0]
                for x in srcs[1:]:
                    acc = oracle.reduce3(op, dtype, x, acc) if s.flags & FOLD_REVERSE else \
                        oracle.reduce3(op, dtype, acc, x)
            space(r, s.flags & DST_ARENA)[s.dst_off + a0:s.dst_off + a1] = acc
        else:
            raise ProtocolError(f"unknown step kind {K}")
    for key in sent:
        if key[:3] in lag_per_run:
            if sent[key] != lagged.get(key, 0):
                raise ProtocolError(f"{key}: {sent[key]} credits sent, {lagged.get(key, 0)} awaited")
            continue
        if sent[key] != consumed.get(key, 0):
            raise ProtocolError(f"{key}: {sent[key]} sent, {consumed.get(key, 0)} consumed")
    if arenas_out is not None:
        arenas_out[:] = arena
    return np.array([[user[r][j] for j in range(k)] for r in range(P)])


INTERP_MAX_STEPS = 512  # gloo_amd/include/gloo_amd/signal.h kInterpMaxSteps
MAX_SRCS = 8            # include/gloo_amd.h GLOO_HIP_MAX_SRCS


def sliced_interp_steps(algo, P, n, rank, k=1, nin=0, recv=None, elem_size=4, max_seg=0):
    """Python statement of executor_modes.cc slicedInterpSteps: an upper bound on the
    device step list buildInterp() emits for `rank`'s sliced plan.  A rank
    proposes slicing only when this is <= INTERP_MAX_STEPS."""
    steps, _ = get_plan(algo, rank, P, n, k, recv, nin=nin, elem_size=elem_size, max_seg=max_seg)
    cuts = user_cuts(steps)
    total = 0
    for t in steps:
        K = t.kind
        if K in (KIND["DECL_RECV"], KIND["WAIT_SEND"], KIND["FOLD_SRC"]):
            continue
        if K == KIND["LOCAL_REDUCE"]:
            srcs = max(1, nin if t.flags & FROM_INPUTS else k)
            per = 1 if srcs <= MAX_SRCS else 1 + (srcs - MAX_SRCS + MAX_SRCS - 2) // (MAX_SRCS - 1)
            total += len(cut_range(cuts, t.dst_off, t.length)) * per
        elif K == KIND["LOCAL_BCAST"]:
            total += len(cut_range(cuts, t.dst_off, t.length)) * max(0, k - 1)
        else:
            total += 1
    return total
