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
            ring_chunked_mesh=6, allreduce_bcube=7, reduce=8)
MESH = 0x100  # algo | MESH: the derived mesh plan (gloo_amd/csrc/mesh.cc)
ALGO.update({"mesh_" + k: v | MESH for k, v in list(ALGO.items()) if v < 5 or v in (5, 7, 8)})
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


def simulate(algo, op, dtype, inputs, recv=None, seed=0, ins=None, max_seg=0, runs=1):
    """inputs: [P][k][n] array of the dtype's storage type (the outputs'
    initial contents); ins: optional [P][kin][n] separate inputs (new-style
    allreduce).  runs > 1 executes the plan back to back that many times
    (each run reduces the previous run's outputs), with no barrier between
    runs, as repeated Algorithm::run() calls do.  Returns the outputs."""
    P, k, n = inputs.shape
    nin = 0 if ins is None else ins.shape[1]
    es = inputs.dtype.itemsize
    plans = [get_plan(algo, r, P, n, k, recv, nin=nin, elem_size=es, max_seg=max_seg) for r in range(P)]
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
    regions = {}
    for r, (steps, _) in enumerate(plans):
        for s in steps:
            if s.kind == KIND["DECL_RECV"]:
                key = (s.peer, r, s.slot)
                if key in regions:
                    raise ProtocolError(f"region {key} declared twice")
                regions[key] = (s.dst_off, s.length)
    sent, consumed, lagged = {}, {}, {}
    pending = [[] for _ in range(P)]  # FOLD sources, read when the FOLD executes
    pc = [0] * P
    rng = random.Random(seed)

    def space(r, is_arena):
        return arena[r] if is_arena else user[r][0]

    def runnable(r):
        steps = plans[r][0]
        if pc[r] >= len(steps):
            return False
        s = steps[pc[r]]
        if s.kind == KIND["WAIT_NOTIFY"] and s.flags & PREV_RUN:
            # the i-th such wait is met by the previous run's credits
            key = (s.peer, r, s.slot)
            return sent.get(key, 0) >= lagged.get(key, 0) + 1 - lag_per_run[key]
        if s.kind in (KIND["WAIT_RECV"], KIND["WAIT_NOTIFY"]):
            key = (s.peer, r, s.slot)
            return sent.get(key, 0) > consumed.get(key, 0)
        return True

    while True:
        ready = [r for r in range(P) if runnable(r)]
        if not ready:
            if all(pc[r] >= len(plans[r][0]) for r in range(P)):
                break
            raise ProtocolError(f"deadlock at pcs {pc}")
        r = rng.choice(ready)
        s = plans[r][0][pc[r]]
        pc[r] += 1
        K = s.kind
        if K == KIND["DECL_RECV"] or K == KIND["WAIT_SEND"]:
            continue
        if K == KIND["WAIT_NOTIFY"] and s.flags & PREV_RUN:
            key = (s.peer, r, s.slot)
            lagged[key] = lagged.get(key, 0) + 1
            continue
        if K == KIND["SEND"]:
            key = (r, s.peer, s.slot)
            if key not in regions:
                raise ProtocolError(f"send to undeclared region {key}")
            if sent.get(key, 0) > consumed.get(key, 0):
                raise ProtocolError(f"send {key} overwrites an unconsumed message")
            roff, cap = regions[key]
            if s.length > cap:
                raise ProtocolError(f"send {key} of {s.length} exceeds region {cap}")
            src = ins[r, 0] if s.flags & FROM_INPUTS else space(r, s.flags & SRC_ARENA)
            arena[s.peer][roff:roff + s.length] = src[s.src_off:s.src_off + s.length]
            sent[key] = sent.get(key, 0) + 1
        elif K in (KIND["WAIT_RECV"], KIND["WAIT_NOTIFY"]):
            key = (s.peer, r, s.slot)
            consumed[key] = consumed.get(key, 0) + 1
        elif K == KIND["NOTIFY"]:
            key = (r, s.peer, s.slot)
            sent[key] = sent.get(key, 0) + 1
        elif K == KIND["REDUCE"]:
            dst = user[r][0]
            # FROM_INPUTS: out = in op inbox (gloo::reduce, gloo/reduce.cc:180-184)
            a = (ins[r, 0] if s.flags & FROM_INPUTS else dst)[s.dst_off:s.dst_off + s.length]
            b = arena[r][s.src_off:s.src_off + s.length]
            dst[s.dst_off:s.dst_off + s.length] = oracle.reduce3(op, dtype, a, b)
        elif K == KIND["COPY"]:
            src = space(r, s.flags & SRC_ARENA)
            dst = space(r, s.flags & DST_ARENA)
            dst[s.dst_off:s.dst_off + s.length] = src[s.src_off:s.src_off + s.length].copy()
        elif K == KIND["LOCAL_REDUCE"]:
            lo, hi = s.dst_off, s.dst_off + s.length
            out0 = user[r][0]
            if s.flags & FROM_INPUTS:
                if nin == 1:
                    out0[lo:hi] = ins[r, 0, lo:hi]
                else:
                    out0[lo:hi] = oracle.reduce3(op, dtype, ins[r, 0, lo:hi], ins[r, 1, lo:hi])
                    for j in range(2, nin):
                        out0[lo:hi] = oracle.reduce3(op, dtype, out0[lo:hi], ins[r, j, lo:hi])
            else:
                for j in range(1, k):
                    out0[lo:hi] = oracle.reduce3(op, dtype, out0[lo:hi], user[r][j][lo:hi])
        elif K == KIND["LOCAL_BCAST"]:
            lo, hi = s.dst_off, s.dst_off + s.length
            for j in range(1, k):
                user[r][j][lo:hi] = user[r][0][lo:hi]
        elif K == KIND["FOLD_SRC"]:
            pending[r].append((s.flags, s.src_off))
        elif K == KIND["FOLD"]:
            srcs = [(ins[r, 0] if f & FROM_INPUTS else space(r, f & SRC_ARENA))[o:o + s.length].copy()
                    for f, o in pending[r]]
            pending[r] = []
            if s.flags & FOLD_TREE:
                while len(srcs) > 1:
                    srcs = [oracle.reduce3(op, dtype, srcs[2 * j], srcs[2 * j + 1]) for j in range(len(srcs) // 2)]
                acc = srcs[0]
            else:
                acc = srcs[0]
                for x in srcs[1:]:
                    acc = oracle.reduce3(op, dtype, x, acc) if s.flags & FOLD_REVERSE else \
                        oracle.reduce3(op, dtype, acc, x)
            space(r, s.flags & DST_ARENA)[s.dst_off:s.dst_off + s.length] = acc
        else:
            raise ProtocolError(f"unknown step kind {K}")
    for key in sent:
        if key in lag_per_run:
            if sent[key] != lagged.get(key, 0):
                raise ProtocolError(f"{key}: {sent[key]} credits sent, {lagged.get(key, 0)} awaited")
            continue
        if sent[key] != consumed.get(key, 0):
            raise ProtocolError(f"{key}: {sent[key]} sent, {consumed.get(key, 0)} consumed")
    return np.array([[user[r][j] for j in range(k)] for r in range(P)])
