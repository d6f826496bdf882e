"""One rank of a mode-matrix cell (tests/mode_matrix.py) — TEST
INFRASTRUCTURE.  Imported by tests/test_mode_matrix_gpu.py for ranks as
threads, run as a script for ranks as processes:

    python mode_matrix_rank.py RANK P STORE CASE COMPLETION WORKSPACE OUT

Three runs of the golden case's algorithm, the buffer reset to the rank's
input before each; writes OUT (json: each run's output bytes as hex, and
mode() after each run)."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for _p in (ROOT, HERE):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import gloo_amd  # noqa: E402
import hip_rt  # noqa: E402

RUNS = 3


def run_rank(rank, P, store, case, completion, workspace, timeout_ms=60000):
    """With torch already imported (ranks as threads inside pytest) the
    buffers and the caller's stream are torch's, so the process keeps one HIP
    runtime; a rank process uses hip_rt without torch."""
    g = np.load(os.path.join(ROOT, "tests", "golden", "sched_golden.npz"))
    algo, op, dtype = case.split("/")[:3]
    x = g[case + "/in"][rank, 0]
    torch = sys.modules.get("torch")
    if torch is not None:
        torch.cuda.set_device(0)
        src = torch.from_numpy(x.view(np.uint8).copy()).to("cuda:0")
        t = torch.empty_like(src)
        buf = t.data_ptr()
        ts = torch.cuda.Stream() if completion == "caller" else None
        stream = ts.cuda_stream if ts is not None else 0

        def reset():
            t.copy_(src)
            torch.cuda.synchronize()

        def read():
            if ts is not None:
                ts.synchronize()
            return t.cpu().numpy().tobytes().hex()
    else:
        hip_rt.set_device(0)
        buf = hip_rt.malloc(x.nbytes)
        stream = hip_rt.stream_create() if completion == "caller" else 0

        def reset():
            hip_rt.h2d(buf, x)  # synchronous

        def read():
            if stream:
                hip_rt.stream_synchronize(stream)
            return hip_rt.d2h(buf, x).tobytes().hex()
    ctx = gloo_amd.Context(rank, P, store, device=0, timeout_ms=timeout_ms)
    a = gloo_amd.Algorithm(ctx, algo, op, dtype, [buf], x.size, stream=stream, workspace=workspace)
    outs, modes = [], []
    for _ in range(RUNS):
        reset()
        a.run()
        outs.append(read())
        modes.append(a.mode())
    a.close()
    ctx.close()
    if torch is None:
        if stream:
            hip_rt.stream_destroy(stream)
        hip_rt.free(buf)
    return {"outs": outs, "modes": modes}


if __name__ == "__main__":
    r, P, store, case, completion, workspace, out = sys.argv[1:8]
    res = run_rank(int(r), int(P), store, case, completion, workspace)
    with open(out, "w") as f:
        json.dump(res, f)
