"""One rank of a batch of golden-schedule jobs (tests/sched_pool.py) — test
infrastructure.  argv: RANK P DIR JOBS_JSON.  Every job is a fresh context
(store file:DIR/s<j>) and one algorithm over the case's input from
tests/golden/sched_golden.npz (bcube_golden.npz for AllreduceBcube), run `runs` times with the buffer reset to the
input before each run; it saves the outputs of every run (o<rank>_<j>.npy),
the mode of every run (m<rank>_<j>.json) or the error (e<rank>_<j>.txt), and
goes on with the next job.  Device memory comes from tests/hip_rt.py, not
torch, so the process starts quickly."""
import json
import os
import sys
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import gloo_amd  # noqa: E402
import hip_rt  # noqa: E402


def main():
    rank, P, d, jobs = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], json.loads(open(sys.argv[4]).read())
    g = np.load(os.path.join(ROOT, "tests", "golden", "sched_golden.npz"))
    gb = np.load(os.path.join(ROOT, "tests", "golden", "bcube_golden.npz"))
    hip_rt.set_device(0)
    for j, job in enumerate(jobs):
        case, runs = job["case"], job["runs"]
        try:
            algo, op, dtype = case.split("/")[:3]
            x = (gb if algo == "bcube" else g)[case + "/in"]
            recv = g[case + "/recv"] if algo == "reduce_scatter" else None
            if algo == "bcube":  # AllreduceBcube: recv_elems = [base] (key .../b<base>/...)
                recv = [int(case.split("/")[4][1:])]
            xr = x[rank] if algo == "reduce_scatter" else x[rank, 0]
            buf = hip_rt.malloc(xr.nbytes)
            ctx = gloo_amd.Context(rank, P, "file:" + os.path.join(d, f"s{j}"), device=0,
                                   timeout_ms=job.get("timeout_ms", 30000))
            a = gloo_amd.Algorithm(ctx, algo, op, dtype, [buf], xr.size, recv_elems=recv)
            outs, modes = [], []
            for _ in range(runs):
                hip_rt.h2d(buf, xr)
                a.run()
                modes.append(a.mode())
                outs.append(hip_rt.d2h(buf, xr))
            a.close()
            ctx.close()
            hip_rt.free(buf)
            np.save(os.path.join(d, f"o{rank}_{j}.npy"), np.array(outs))
            with open(os.path.join(d, f"m{rank}_{j}.json"), "w") as f:
                json.dump(modes, f)
        except Exception:  # noqa: BLE001 — recorded for the test of this job
            with open(os.path.join(d, f"e{rank}_{j}.txt"), "w") as f:
                f.write(traceback.format_exc())


if __name__ == "__main__":
    main()
