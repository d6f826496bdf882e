"""Compare the two reduce-kernel timings of the executor (events around each
step vs device stamps inside the kernels) where they must agree, and where
they may not (events and eager stamps time the same schedule; replay
changes the schedule):

  ring    P ranks as processes on this GPU, ring-chunked mesh plan at n per
          rank — events (eager), stamps with GLOO_AMD_GRAPH=0 (eager),
          stamps replayed.

Usage: python tools/stamp_check.py [P] [log2 n]   (prints JSON lines)
"""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import os, sys, json
sys.path.insert(0, os.environ["GLOO_AMD_ROOT"])
import torch, gloo_amd
rank, size, store, algo, n, k = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], int(sys.argv[5]), int(sys.argv[6])
torch.cuda.set_device(0)
bufs = [torch.ones(n, device="cuda:0") for _ in range(k)]
ctx = gloo_amd.Context(rank, size, store, device=0, timeout_ms=120000)
a = gloo_amd.Algorithm(ctx, algo, "sum", "f32", [b.data_ptr() for b in bufs], n)
mode = int(os.environ["STAMP_MODE"])
a.set_profiling(mode)
rows = []
for it in range(8):
    a.run()
    st = a.stats()
    rows.append({"graph": a.mode()["graph"], "gib_s": st["reduce_bytes"] / st["reduce_s"] / 2**30 if st["reduce_s"] else None,
                 "reduce_us": st["reduce_s"] * 1e6, "reductions": st["reductions"]})
a.close(); ctx.close()
print("RESULT" + json.dumps(rows), flush=True)
'''


def run(P, algo, n, k, mode, graph):
    with tempfile.TemporaryDirectory() as d:
        w = os.path.join(d, "w.py")
        open(w, "w").write(WORKER)
        env = dict(os.environ, GLOO_AMD_ROOT=ROOT, STAMP_MODE=str(mode), GLOO_AMD_GRAPH=graph)
        procs = [subprocess.Popen([sys.executable, w, str(r), str(P), "file:" + os.path.join(d, "s"), algo, str(n),
                                   str(k)], env=env, stdout=subprocess.PIPE, text=True) for r in range(P)]
        outs = [p.communicate(timeout=300)[0] for p in procs]
        if any(p.returncode for p in procs):
            return {"error": [p.returncode for p in procs]}
    res = [json.loads(o.split("RESULT", 1)[1]) for o in outs]
    tail = [rows[3:] for rows in res]  # after capture
    return {"graph_last": [rows[-1]["graph"] for rows in res],
            "gib_s_per_rank": [round(sum(r["gib_s"] or 0 for r in t) / len(t), 1) for t in tail],
            "reduce_us_per_rank": [round(sum(r["reduce_us"] for r in t) / len(t), 1) for t in tail],
            "reductions": res[0][-1]["reductions"]}


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    n = 1 << (int(sys.argv[2]) if len(sys.argv) > 2 else 26)
    cases = [("ring", P, "ring_chunked", n, 1)]
    for name, p, algo, nn, k in cases:
        for label, mode, graph in (("events", 1, "auto"), ("stamps_eager", 2, "0"), ("stamps_replayed", 2, "auto")):
            out = {"case": name, "P": p, "n": nn, "k": k, "timing": label, **run(p, algo, nn, k, mode, graph)}
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
