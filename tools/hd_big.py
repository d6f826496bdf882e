"""DIAGNOSIS ONLY: halving-doubling fp32 sum at a large size per rank, P rank
processes on the box's GPU(s), timing construction and each run, printing
progress as it goes (closed-form check: element j of rank r holds
(j % 1024) * P + r).

  python tools/hd_big.py P N [RUNS]     (env passes through: GLOO_AMD_MESH=0 ...)
"""
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r"""
import os, sys, time
sys.path.insert(0, os.environ["GLOO_AMD_ROOT"])
import torch, gloo_amd
rank, P, store, n, runs = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
dev = rank % torch.cuda.device_count()
torch.cuda.set_device(dev)
t0 = time.time()
def say(m):
    print(f"[r{rank} {time.time() - t0:7.2f}s] {m}", file=sys.stderr, flush=True)
ctx = gloo_amd.Context(rank, P, store, device=dev, timeout_ms=60000)
j = torch.arange(n, device=f"cuda:{dev}", dtype=torch.int64) % 1024
src = (j * P + rank).float()
want = (j * P * P + P * (P - 1) // 2).float()
del j
buf = torch.empty_like(src)
say("constructing")
a = gloo_amd.Algorithm(ctx, "halving_doubling", "sum", "f32", [buf.data_ptr()], n)
say(f"constructed {a.mode()}")
for it in range(runs):
    buf.copy_(src)
    torch.cuda.synchronize()
    t = time.time()
    a.run()
    say(f"run {it}: {(time.time() - t) * 1e3:.1f} ms, equal={bool(torch.equal(buf, want))}, {a.mode()}")
a.close()
ctx.close()
say("done")
"""


def main():
    P, n = int(sys.argv[1]), int(sys.argv[2])
    runs = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    with tempfile.TemporaryDirectory() as d:
        w = os.path.join(d, "w.py")
        open(w, "w").write(WORKER)
        env = dict(os.environ, GLOO_AMD_ROOT=ROOT)
        procs = [subprocess.Popen([sys.executable, w, str(r), str(P), "file:" + os.path.join(d, "s"), str(n), str(runs)],
                                  env=env) for r in range(P)]
        t0 = time.time()
        while any(p.poll() is None for p in procs):
            if time.time() - t0 > float(os.environ.get("HD_BIG_TIMEOUT", "150")):
                print("hd_big: timeout, killing", flush=True)
                for p in procs:
                    p.kill()
                sys.exit(3)
            time.sleep(0.5)
        print("hd_big: exit codes", [p.returncode for p in procs], flush=True)
        sys.exit(max(p.returncode for p in procs))


if __name__ == "__main__":
    main()
