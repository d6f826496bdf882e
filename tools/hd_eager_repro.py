#!/usr/bin/env python3
"""Two rank processes on one GPU replaying bench.py's N>1 HD sweep order
(a fresh context + algorithm per size, variants back to back) to find which
executor the 'invalid argument' of an eager SEND copy comes from
(profiles/round2/r2zx_bench_n2_one_gpu_rehearsal.json).  One JSON line per
(rank, variant, size).

usage: hd_eager_repro.py            (spawns both ranks)
"""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

VARIANTS = [("mesh", {}), ("mesh_memcpy_forked", {"GLOO_AMD_COPY": "memcpy"}),
            ("mesh_eager", {"GLOO_AMD_GRAPH": "0", "GLOO_AMD_INTERP": "0"}),
            ("reference_route_eager", {"GLOO_AMD_MESH": "0", "GLOO_AMD_GRAPH": "0", "GLOO_AMD_INTERP": "0"})]
SIZES = (1 << 10, 64 << 10, 1 << 20, 64 << 20)


def rank_main(rank, world, d, with_config3):
    import torch
    import gloo_amd as hip
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    if with_config3:
        # bench.py's config-3 section first: 2 x 256 MiB ring-chunked executors
        for k, env in enumerate([{}, {"GLOO_AMD_RING_MESH": "0"}]):
            old = {e: os.environ.get(e) for e in env}
            os.environ.update(env)
            b = torch.ones(1 << 26, device=dev)
            ctx = hip.Context(rank, world, f"file:{d}/c3_{k}", device=0, timeout_ms=60000)
            a = hip.Algorithm(ctx, "ring_chunked", "sum", "f32", [b.data_ptr()], b.numel())
            for _ in range(3):
                a.run()
            a.close()
            ctx.close()
            del b
            for e, v in old.items():
                if v is None:
                    os.environ.pop(e, None)
                else:
                    os.environ[e] = v
    for name, env in VARIANTS:
        old = {e: os.environ.get(e) for e in env}
        os.environ.update(env)
        for nbytes in SIZES:
            m = nbytes // 4
            rec = {"rank": rank, "variant": name, "bytes": nbytes}
            try:
                b2 = torch.full((m,), float(rank + 1), device=dev)
                torch.cuda.synchronize(dev)
                ctx2 = hip.Context(rank, world, f"file:{d}/hd_{name}_{nbytes}", device=0, timeout_ms=60000)
                a2 = hip.Algorithm(ctx2, "halving_doubling", "sum", "f32", [b2.data_ptr()], m)
                a2.run()
                rec["ok"] = bool((b2 == world * (world + 1) / 2).all())
                for _ in range(3):
                    a2.run()
                torch.cuda.synchronize(dev)
                rec["mode"] = a2.mode()
                a2.close()
                ctx2.close()
            except Exception as e:  # noqa: BLE001
                rec["error"] = repr(e)[:600]
            print(json.dumps(rec), flush=True)
            if "error" in rec:
                return 1
        for e, v in old.items():
            if v is None:
                os.environ.pop(e, None)
            else:
                os.environ[e] = v
    return 0


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "rank":
        sys.exit(rank_main(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5] == "1"))
    with_c3 = "--config3" in sys.argv
    with tempfile.TemporaryDirectory() as d:
        ps = [subprocess.Popen([sys.executable, __file__, "rank", str(r), "2", d, "1" if with_c3 else "0"])
              for r in range(2)]
        rcs = [p.wait(timeout=240) for p in ps]
    sys.exit(max(rcs))


if __name__ == "__main__":
    main()
