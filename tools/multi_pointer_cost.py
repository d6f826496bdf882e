"""MEASUREMENT: what pipelineBroadcastAndReduce could hide (VERDICT r5
"missing" 3).

The reference's CudaAllreduceHalvingDoubling with several device pointers per
rank can pipeline its local reduce and broadcast with the exchange
(pipelineBroadcastAndReduce, gloo/cuda_allreduce_halving_doubling.cc:253-279,
376-394).  This library accepts the flag and runs the local parts as one
fused pass each (a k-source left fold before the exchange, a broadcast after
it).  The most a pipeline could save is the time of those local passes, so
this times the same halving-doubling allreduce (fp32 sum, n elements per
pointer, P rank processes on the box's GPU) with k = 1 pointer and with k
pointers per rank: (t_k - t_1) / t_k bounds the pipeline's gain.

    python tools/multi_pointer_cost.py RANK P STORE_DIR N K ITERS
(launched by tools/multi_pointer_cost.sh); rank 0 prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import gloo_amd  # noqa: E402
import hip_rt  # noqa: E402


def main():
    rank, P, d, n, K, iters = (int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4]),
                               int(sys.argv[5]), int(sys.argv[6]))
    hip_rt.set_device(0)
    ctx = gloo_amd.Context(rank, P, "file:" + d, device=0, timeout_ms=60000)
    out = {"P": P, "n_per_pointer": n, "iters": iters}
    x = np.full(n, 1.0, np.float32)
    for k in (1, K):
        bufs = [hip_rt.malloc(4 * n) for _ in range(k)]
        for b in bufs:
            hip_rt.h2d(b, x)
        a = gloo_amd.Algorithm(ctx, "halving_doubling", "sum", "f32", bufs, n)
        for _ in range(3):
            a.run()
        ctx_barrier = gloo_amd.Algorithm(ctx, "halving_doubling", "sum", "f32", [bufs[0]], 1)
        ts = []
        for _ in range(iters):
            ctx_barrier.run()  # line the ranks up
            t0 = time.perf_counter()
            a.run()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        out["k%d_us_p50" % k] = round(ts[len(ts) // 2] * 1e6, 1)
        y = hip_rt.d2h(bufs[-1], x)
        out["k%d_finite" % k] = bool(np.isfinite(y).all())
        ctx_barrier.close()
        a.close()
        for b in bufs:
            hip_rt.free(b)
    out["K"] = K
    out["local_share_bound"] = round((out["k%d_us_p50" % K] - out["k1_us_p50"]) / out["k%d_us_p50" % K], 4)
    ctx.close()
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
