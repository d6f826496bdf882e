"""DIAGNOSIS: GPUTEST_r05's red case as an A/B rate, not a rerun of the suite.

The test that failed once (tests/test_newstyle_gpu.py::test_bcube_threads_golden,
case bcube/sum/f32/P12/i0/o1/n10/s0 on the reference route) makes twelve rank
threads on one GPU call gloo::allreduce BCUBE twice, the second call on
rebound buffers.  This repeats exactly that `iters` times per golden case and
counts wrong results by call, for whichever library build GLOO_AMD_LIB names
(the product's, with fine-grained inboxes, or an A/B build that keeps the
round-5 coarse-grained inbox for same-GPU thread ranks),
or for another tree's package entirely (GLOO_AMD_PKG_ROOT: a directory holding
a `gloo_amd/` package, e.g. round 5's as the driver ran it).

    python tools/bcube_threads_stress.py ITERS [case ...]

One JSON line per case: iterations, wrong results per call, the fine_arena
mode the executor reported, and the first wrong value seen."""
import json
import os
import sys
import threading
import uuid

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("GLOO_AMD_PKG_ROOT") or ROOT)

import numpy as np  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden", "newstyle_golden.npz")


def main():
    import torch
    import gloo_amd
    os.environ["GLOO_AMD_MESH"] = "0"
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    cases = sys.argv[2:] or ["bcube/sum/f32/P12/i0/o1/n10/s0", "bcube/sum/f32/P12/i0/o1/n4099/s0"]
    z = np.load(GOLDEN)
    for case in cases:
        parts = case.split("/")
        op, dtype, P, n = parts[1], parts[2], int(parts[3][1:]), int(parts[6][1:])
        init, want = z[case + "/init"], z[case + "/out"]
        wrong = [0, 0]
        fine = set()
        first = []
        lock = threading.Lock()
        for it in range(iters):
            url = "mem:" + uuid.uuid4().hex
            errors = []

            def body(r):
                try:
                    torch.cuda.set_device(0)
                    ctx = gloo_amd.Context(r, P, url, device=0, timeout_ms=60000)
                    for rep in range(2):
                        out = torch.from_numpy(init[r, 0].view(np.uint8).copy()).to("cuda:0")
                        torch.cuda.synchronize()
                        gloo_amd.allreduce(ctx, [out.data_ptr()], n, dtype, op, algorithm="bcube")
                        y = out.cpu().numpy().view(init.dtype)
                        m = ctx.last_mode()
                        with lock:
                            fine.add(bool(m.get("fine_arena")))
                            if y.view(np.uint8).tobytes() != want.view(np.uint8).tobytes():
                                wrong[rep] += 1
                                if not first:
                                    k = int(np.flatnonzero(y != want)[0])
                                    first.append({"iter": it, "rank": r, "call": rep, "index": k,
                                                  "got": float(y[k]), "want": float(want[k])})
                    ctx.close()
                except Exception as e:  # noqa: BLE001
                    errors.append((r, repr(e)))

            ts = [threading.Thread(target=body, args=(r,)) for r in range(P)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            if errors:
                print(json.dumps({"case": case, "iter": it, "errors": errors[:3]}), flush=True)
                sys.exit(1)
        print(json.dumps({"case": case, "lib": os.path.relpath(gloo_amd.LIB_PATH, ROOT), "iterations": iters,
                          "results_per_call": iters * P, "wrong_first_call": wrong[0],
                          "wrong_second_call": wrong[1], "fine_arena": sorted(fine), "first_wrong": first}),
              flush=True)


if __name__ == "__main__":
    main()
