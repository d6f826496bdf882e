"""Run ring-chunked allreduce variants back to back in the same rank
processes, as bench.py's xgmi_allreduce section does (a new Context and
Algorithm per variant, GLOO_AMD_COPY / GLOO_AMD_RING_MESH set around the
construction), and check every element of each variant's first run against
the closed form of gloo/test/base_test.h:184-236.

Usage: [SEQ_RANDOM=1] python tools/variant_sequence_check.py P log2n seq [seq ...]
  SEQ_RANDOM=1: N(0,1) inputs from seed (7, rank), as bench.py uses, checked
  against the reference's ring fold order (computed on the host)
  seq = comma-separated variants, each <copy>-<mesh|ring>, e.g.
        auto-mesh,memcpy-ring,kernel-ring
Prints one JSON line per sequence: bad elements per variant per rank.
"""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import json, os, sys
sys.path.insert(0, os.environ["GLOO_AMD_ROOT"])
import torch, gloo_amd
rank, size, storedir, n, seq = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), sys.argv[5].split(",")
torch.cuda.set_device(0)
dev = torch.device("cuda:0")
random_data = os.environ.get("SEQ_RANDOM") == "1"
if random_data:
    import numpy as np
    xs = [np.random.default_rng([7, r]).standard_normal(n, dtype=np.float32) for r in range(size)]
    chunks = 2 * size
    cs = max(256, (n + chunks - 1) // chunks)
    q = (np.arange(n) // cs) // 2  # the rank that starts each chunk pair's fold
    acc = np.choose(q % size, xs).astype(np.float32) if size > 1 else xs[0]
    for j in range(1, size):
        acc = np.choose((q + j) % size, xs).astype(np.float32) + acc
    want = torch.from_numpy(acc).to(dev)
    mine = torch.from_numpy(xs[rank]).to(dev)
    del xs, acc, q
else:
    want = (torch.arange(n, device=dev, dtype=torch.int64) % 1024 * size * size + size * (size - 1) // 2).float()
    mine = ((torch.arange(n, device=dev, dtype=torch.int64) % 1024) * size + rank).float()
out = []
for k, v in enumerate(seq):
    copy, route = v.split("-")
    os.environ["GLOO_AMD_COPY"] = copy
    os.environ["GLOO_AMD_RING_MESH"] = "1" if route == "mesh" else "0"
    buf = mine.clone()
    torch.cuda.synchronize()
    ctx = gloo_amd.Context(rank, size, "file:%s/v%d" % (storedir, k), device=0, timeout_ms=60000)
    a = gloo_amd.Algorithm(ctx, "ring_chunked", "sum", "f32", [buf.data_ptr()], n)
    a.run()
    torch.cuda.synchronize()
    bad = int((buf != want).sum())
    extra = []
    # the bench's later runs on the same algorithm: timed, events, stamps
    for prof, runs in ((0, 5), (1, 3), (2, 7)):
        a.set_profiling(prof)
        for _ in range(runs):
            buf.copy_(mine)
            torch.cuda.synchronize()
            a.run()
            torch.cuda.synchronize()
            extra.append(int((buf != want).sum()))
    a.set_profiling(0)
    a.close(); ctx.close()
    del buf
    out.append({"variant": v, "first_bad": bad, "later_bad": extra})
print("RESULT" + json.dumps(out), flush=True)
'''


def main():
    P, n = int(sys.argv[1]), 1 << int(sys.argv[2])
    for seq in sys.argv[3:]:
        with tempfile.TemporaryDirectory() as d:
            w = os.path.join(d, "w.py")
            open(w, "w").write(WORKER)
            env = dict(os.environ, GLOO_AMD_ROOT=ROOT)
            procs = [subprocess.Popen([sys.executable, w, str(r), str(P), d, str(n), seq], env=env,
                                      stdout=subprocess.PIPE, text=True) for r in range(P)]
            outs = [p.communicate(timeout=300)[0] for p in procs]
        if any(p.returncode for p in procs):
            print(json.dumps({"seq": seq, "error": [p.returncode for p in procs]}), flush=True)
            continue
        res = [json.loads(o.split("RESULT", 1)[1]) for o in outs]
        print(json.dumps({"seq": seq, "P": P, "n": n, "ranks": res}), flush=True)


if __name__ == "__main__":
    main()
