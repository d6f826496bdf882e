"""DIAGNOSIS ONLY: which use of an executor's IPC import leaves it alive after
hipIpcCloseMemHandle, so that the next import of a byte-identical handle
(the peer's next same-size arena at the same address) maps the OLD pages.

Two rank processes on one GPU (torch.distributed gloo for the barriers).
Executor A (ring-chunked fp32 sum, --mib per rank, the ring route) is built
with the env of --first, run --runs times (graph replay from run 3 unless
GLOO_AMD_GRAPH=0), optionally with profiling, destroyed; executor B (the
same size, kernel copies) is built next.  With GLOO_AMD_IPC_POOL=0 the
peer's arena of B comes back at A's address; B's construction reports
whether its imports showed the peer's nonce (the executor's check), with no
retry.  One JSON line per rank.

  python tools/ipc_bisect.py --first COPY=memcpy,GRAPH=1 --runs 3 --profile 0
"""
import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def body(rank, world, args, store_dir):
    import numpy as np
    import torch
    import torch.distributed as dist
    import gloo_amd as hip

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n = args.mib * (1 << 20) // 4
    buf = torch.from_numpy(np.random.default_rng([7, rank]).standard_normal(n, dtype=np.float32)).to(dev)
    torch.cuda.synchronize(dev)
    env = dict(kv.split("=") for kv in args.first.split(",") if kv)
    out = {"rank": rank, "first": env}

    def with_env(e, fn):
        old = {k: os.environ.get(k) for k in e}
        os.environ.update(e)
        try:
            return fn()
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

    def first():
        ctx = hip.Context(rank, world, "file:%s/a" % store_dir, device=0, timeout_ms=60000)
        a = hip.Algorithm(ctx, "ring_chunked", "sum", "f32", [buf.data_ptr()], n)
        for _ in range(args.runs):
            dist.barrier()
            a.run()
        if args.profile:
            a.set_profiling(args.profile)
            for _ in range(2):
                dist.barrier()
                a.run()
            a.set_profiling(0)
        out["first_mode"] = a.mode()
        a.close()
        ctx.close()

    with_env({"GLOO_AMD_" + k: v for k, v in env.items()}, first)
    dist.barrier()

    def second():
        ctx = hip.Context(rank, world, "file:%s/b" % store_dir, device=0, timeout_ms=60000)
        try:
            a = hip.Algorithm(ctx, "ring_chunked", "sum", "f32", [buf.data_ptr()], n)
            a.run()
            out["second"] = "ok"
            a.close()
        except Exception as e:  # noqa: BLE001
            out["second"] = repr(e)[:300]
        ctx.close()

    with_env({"GLOO_AMD_COPY": "kernel"}, second)
    out["stale"] = "does not show its contents" in out.get("second", "")
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--first", default="COPY=memcpy")
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--profile", type=int, default=0)
    ap.add_argument("--mib", type=int, default=256)
    args = ap.parse_args()
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = [tempfile.mkdtemp(prefix="ipcb_")] if rank == 0 else [None]
    dist.broadcast_object_list(d, src=0)
    body(rank, world, args, d[0])
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
