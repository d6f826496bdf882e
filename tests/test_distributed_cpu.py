"""CPU, multi-process: the N>1 path without a GPU.

1. The per-rank plans from gloo_hip_plan executed by separate processes that
   exchange messages over torch.distributed's gloo backend (world_size 2 and
   3, 127.0.0.1), reductions by the oracle restatement of gloo/math.h; results
   compared byte for byte with the reference's schedule goldens.
2. The C++ Context rendezvous (FileStore + shared-memory control block,
   gloo_amd/csrc/context.cc) created and torn down by separate processes.
"""
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PLAN_WORKER = r'''
import os, sys
sys.path.insert(0, os.environ["GLOO_AMD_ROOT"]); sys.path.insert(0, os.path.join(os.environ["GLOO_AMD_ROOT"], "tests"))
import numpy as np, torch, torch.distributed as dist
import oracle
from plan_sim import KIND, SRC_ARENA, DST_ARENA, FOLD_REVERSE, get_plan
rank, size, port, case, outdir = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], sys.argv[5]
plan_algo = sys.argv[6] if len(sys.argv) > 6 else None
dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=size)
algo, op, dtype = case.split("/")[:3]
newstyle = algo in ("bcube", "reduce")
g = np.load(os.path.join(os.environ["GLOO_AMD_ROOT"], "tests", "golden",
                         "newstyle_golden.npz" if newstyle else "sched_golden.npz"))
ins = None
if newstyle:
    parts = case.split("/")
    x = g[case + "/init"]
    ins = g[case + "/in"][rank] if case + "/in" in g.files else None
    if algo == "reduce":
        recv = np.array([int(parts[6][1:])], np.int32)
        seg = int(parts[7][1:])
    else:
        recv, seg = None, int(parts[7][1:])
else:
    x = g[case + "/in"]
    recv = g[case + "/recv"] if algo == "reduce_scatter" else None
    seg = 0
if algo == "reduce_scatter":
    x = x[:, None, :]
P, k, n = x.shape
plan_name = plan_algo or {"bcube": "allreduce_bcube"}.get(algo, algo)
steps, arena_n = get_plan(plan_name, rank, P, n, k, recv, nin=0 if ins is None else ins.shape[0],
                          elem_size=x.dtype.itemsize, max_seg=seg)
fold = []
user = [x[rank, j].copy() for j in range(k)]
FROM_INPUTS = 4
arena = np.zeros(max(1, arena_n), dtype=x.dtype)
regions = {(s.peer, s.slot): (s.dst_off, s.length) for s in steps if s.kind == KIND["DECL_RECV"]}
as_t = lambda a: torch.from_numpy(a.view(np.uint8).copy())
pending = []
for s in steps:
    K = s.kind
    if K == KIND["SEND"]:
        src = ins[0] if s.flags & FROM_INPUTS else arena if s.flags & SRC_ARENA else user[0]
        payload = src[s.src_off:s.src_off + s.length]
        pending.append(dist.isend(torch.tensor([s.length], dtype=torch.int64), s.peer, tag=10 * s.slot))
        pending.append(dist.isend(as_t(payload), s.peer, tag=10 * s.slot + 1))
    elif K == KIND["WAIT_RECV"]:
        hdr = torch.zeros(1, dtype=torch.int64)
        dist.recv(hdr, s.peer, tag=10 * s.slot)
        ln = int(hdr[0]); off, cap = regions[(s.peer, s.slot)]
        assert ln <= cap
        buf = torch.zeros(ln * x.dtype.itemsize, dtype=torch.uint8)
        dist.recv(buf, s.peer, tag=10 * s.slot + 1)
        arena[off:off + ln] = buf.numpy().view(x.dtype)
    elif K == KIND["NOTIFY"]:
        pending.append(dist.isend(torch.zeros(1), s.peer, tag=10 * s.slot + 5))
    elif K == KIND["WAIT_NOTIFY"]:
        dist.recv(torch.zeros(1), s.peer, tag=10 * s.slot + 5)
    elif K == KIND["REDUCE"]:
        d = (ins[0] if s.flags & FROM_INPUTS else user[0])[s.dst_off:s.dst_off + s.length]
        user[0][s.dst_off:s.dst_off + s.length] = oracle.reduce3(op, dtype, d, arena[s.src_off:s.src_off + s.length])
    elif K == KIND["COPY"]:
        src = arena if s.flags & SRC_ARENA else user[0]
        dst = arena if s.flags & DST_ARENA else user[0]
        dst[s.dst_off:s.dst_off + s.length] = src[s.src_off:s.src_off + s.length].copy()
    elif K == KIND["LOCAL_REDUCE"]:
        lo, hi = s.dst_off, s.dst_off + s.length
        if s.flags & FROM_INPUTS:
            acc = ins[0][lo:hi].copy()
            for j in range(1, ins.shape[0]):
                acc = oracle.reduce3(op, dtype, acc, ins[j][lo:hi])
            user[0][lo:hi] = acc
        else:
            for j in range(1, k):
                user[0][lo:hi] = oracle.reduce3(op, dtype, user[0][lo:hi], user[j][lo:hi])
    elif K == KIND["LOCAL_BCAST"]:
        for j in range(1, k):
            user[j][s.dst_off:s.dst_off + s.length] = user[0][s.dst_off:s.dst_off + s.length]
    elif K == KIND["FOLD_SRC"]:
        fold.append((arena if s.flags & SRC_ARENA else user[0])[s.src_off:s.src_off + s.length].copy())
    elif K == KIND["FOLD"]:
        acc = fold[0]
        for v in fold[1:]:
            acc = oracle.reduce3(op, dtype, v, acc) if s.flags & FOLD_REVERSE else oracle.reduce3(op, dtype, acc, v)
        user[0][s.dst_off:s.dst_off + s.length] = acc
        fold = []
for p in pending:
    p.wait()
dist.barrier()
np.save(os.path.join(outdir, f"out{rank}.npy"), np.array(user))
dist.destroy_process_group()
'''


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


CASES = [("ring_chunked/sum/f32/P2/k1/n1000", None), ("halving_doubling/sum/f32/P2/k1/n1000", None),
         ("halving_doubling/sum/f32/P3/k1/n1000", None), ("ring_chunked/sum/f32/P3/k2/n1000", None),
         ("reduce_scatter/sum/f32/P2/n100", None), ("reduce_scatter/sum/f32/P3/n10007", None),
         ("ring/sum/f32/P3/k1/n1000", None),
         # the reference ring's bytes from the mesh plan (two all-to-all hops)
         ("ring_chunked/sum/f32/P3/k2/n1000", "ring_chunked_mesh"),
         ("ring_chunked/max/f32/P5/k1/n999", "ring_chunked_mesh"),
         # the pipelined ring route: three inboxes, fused reduce + send rounds
         ("ring_chunked/sum/f32/P2/k1/n1000", "ring_chunked_pipe"),
         ("ring_chunked/sum/f32/P3/k2/n1000", "ring_chunked_pipe"),
         # new-style gloo::allreduce BCUBE and gloo::reduce (tests/golden/newstyle_golden.npz)
         ("bcube/sum/f32/P2/i0/o1/n1000/s0", None), ("bcube/sum/f32/P6/i3/o2/n999/s0", None),
         ("reduce/sum/f32/P3/i0/n1000/r2/s128", None), ("reduce/sum/f32/P5/i1/n4099/r2/s0", None)]


@pytest.mark.parametrize("case,plan_algo", CASES)
def test_plans_over_gloo_processes(golden_sched, case, plan_algo):
    algo = case.split("/")[0]
    if algo in ("bcube", "reduce"):
        golden_sched = np.load(os.path.join(ROOT, "tests", "golden", "newstyle_golden.npz"))
    P = int(case.split("/")[3][1:])
    with tempfile.TemporaryDirectory() as d:
        w = os.path.join(d, "w.py")
        open(w, "w").write(PLAN_WORKER)
        env = dict(os.environ, GLOO_AMD_ROOT=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        port = str(free_port())
        procs = [subprocess.Popen([sys.executable, w, str(r), str(P), port, case, d] +
                                  ([plan_algo] if plan_algo else []), env=env)
                 for r in range(P)]
        assert [p.wait(timeout=240) for p in procs] == [0] * P
        outs = [np.load(os.path.join(d, f"out{r}.npy")) for r in range(P)]
    want = golden_sched[case + "/out"]
    if algo == "reduce_scatter":
        recv = golden_sched[case + "/recv"]
        got = np.concatenate([outs[r][0, :recv[r]] for r in range(P)])
        assert (got.view(np.uint8) == want.view(np.uint8)).all()
    elif algo in ("ring", "reduce"):  # rank-specific outputs
        for r in range(P):
            assert (outs[r][0].view(np.uint8) == want[r].view(np.uint8)).all(), r
    else:
        for r in range(P):
            for j in range(outs[r].shape[0]):
                assert (outs[r][j].view(np.uint8) == want.view(np.uint8)).all(), (r, j)


CTX_WORKER = r'''
import os, sys
sys.path.insert(0, os.environ["GLOO_AMD_ROOT"])
import gloo_amd
rank, size, store = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
c = gloo_amd.Context(rank, size, store, device=0, timeout_ms=60000)
c.close()
print("ok", rank)
'''


@pytest.mark.parametrize("P", [2, 4])
def test_context_rendezvous_processes(P):
    """Context::connect across processes needs no GPU: FileStore exchange of
    the control-block name, shm_open/mmap, store barrier."""
    with tempfile.TemporaryDirectory() as d:
        w = os.path.join(d, "c.py")
        open(w, "w").write(CTX_WORKER)
        env = dict(os.environ, GLOO_AMD_ROOT=ROOT)
        procs = [subprocess.Popen([sys.executable, w, str(r), str(P), "file:" + os.path.join(d, "s")], env=env,
                                  stdout=subprocess.PIPE, text=True) for r in range(P)]
        outs = [p.communicate(timeout=120)[0] for p in procs]
        assert [p.returncode for p in procs] == [0] * P
        assert all(f"ok {r}" in outs[r] for r in range(P))


def test_context_timeout_is_io_exception():
    """A rank whose peers never arrive times out with IoException, like
    gloo's context timeout (gloo/context.cc:61-64)."""
    import gloo_amd
    with tempfile.TemporaryDirectory() as d:
        with pytest.raises(gloo_amd.GlooHipError) as e:
            gloo_amd.Context(1, 2, "file:" + os.path.join(d, "s"), device=0, timeout_ms=300)
        assert "timed out" in str(e.value).lower()
