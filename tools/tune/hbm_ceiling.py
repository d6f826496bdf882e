"""MEASUREMENT ONLY: the streaming ceiling of this chip for the config-2
access mix, next to the product kernel, in one session.

tools/tune/libceiling.so (hbm_ceiling.hip; built by gloo_amd/Makefile)
holds streaming kernels with reduce_vec_kernel's access shape and R read /
W write streams of 64 MiB.  Six rotated buffer sets (1.1 GiB) keep every
launch streaming from HBM.  Each pattern: 20 warm-up + 300 back-to-back
launches between two events; bytes = (R + W) x 64 MiB per launch.  The
product's in-place fp32 sum (gloo_hip_reduce) runs in the same loop.
One JSON line per (rep, pattern).
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


def main():
    import torch
    import gloo_amd as hip

    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="libceiling.so", help="libceiling_pre.so: kernel arguments preloaded in SGPRs")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--mib", type=int, default=64, help="MiB per stream per launch")
    ap.add_argument("--only", default="", help="comma list of pattern prefixes")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    L = ctypes.CDLL(os.path.join(HERE, args.lib))
    vp = ctypes.c_void_p
    L.ceil_run.argtypes = [ctypes.c_int, vp, vp, vp, vp, ctypes.c_size_t, vp]
    steps = args.steps
    nbytes = args.mib << 20
    n = nbytes // 4
    nsets = max(6, -(-1152 // (3 * args.mib)))   # >= 1.1 GiB rotated, 4.5x the Infinity Cache
    sets = [tuple(torch.rand(n, device="cuda") for _ in range(3)) for _ in range(nsets)]
    sink = torch.zeros(1024, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream

    pats = []
    for i in range(L.ceil_count()):
        d = (ctypes.c_int * 4)()
        L.ceil_desc(i, d)
        r, w, u, b = list(d)
        if w >= 1000000:  # w = 1 + 1e6 (1 + mode) + 1e3 LDS KiB: stream_x_k (round 6)
            mode, lds = w // 1000000 - 1, (w % 1000000) // 1000
            tag = f"R2W1_x{mode}_lds{lds}"
            w = 1
        elif w >= 100:  # w = 1 + 100 * (1 + LP + 32 SP + 1024 IL): stream_pol_k
            code = w // 100 - 1
            lp, sp, il = code % 32, (code // 32) % 32, code // 1024
            tag = f"R2W1_pol_lp{lp}_sp{sp}{'_il' if il else ''}"
            w = 1
        else:
            lds = w >= 10  # w = 1 + 10 u: the reads go through LDS-DMA (buffer_load ... lds)
            tag = "R2W1_ldsdma" if lds else f"R{r}W{w}"
            w = w % 10
        pats.append((f"{tag}_u{u}_b{b}", i, r + w, False))
        if r == 2 and w == 1:
            pats.append((f"{tag}_inplace_u{u}_b{b}", i, r + w, True))
    pats.append(("product_reduce_inplace", -1, 3, True))
    # the product kernel with the other load order (gloo_hip_set_variant 15:
    # interleaved, the round 3-5 default; before round 6's switch the product
    # was interleaved and variant 15 stream by stream)
    pats.append(("product_reduce_inplace_v15", -16, 3, True))
    # round 6: three workgroups per CU (48 KiB of unused LDS), interleaved / stream by stream
    pats.append(("product_reduce_inplace_v16", -17, 3, True))
    pats.append(("product_reduce_inplace_v17", -18, 3, True))
    if args.only:
        pats = [p for p in pats if p[0].startswith(tuple(args.only.split(",")))]

    def launch(p, j):
        name, i, streams, inplace = p
        a, b, c = sets[j % nsets]
        if i < 0:
            hip.set_variant(-i - 1)
            hip.reduce_ptr("sum", "f32", a.data_ptr(), b.data_ptr(), n, s)
            hip.set_variant(0)
            return
        rc = L.ceil_run(i, (a if inplace else c).data_ptr(), a.data_ptr(), b.data_ptr(), sink.data_ptr(), nbytes, s)
        if rc:
            raise RuntimeError(f"{name}: launch failed {rc}")

    # correctness of the 3-operand and copy shapes
    a, b, c = sets[0]
    for p in pats:
        name, i, streams, inplace = p
        if i >= 0 and name.startswith(("R2W1_u", "R1W1", "R2W1_ldsdma_u", "R2W1_pol", "R2W1_x")):
            L.ceil_run(i, c.data_ptr(), a.data_ptr(), b.data_ptr(), sink.data_ptr(), nbytes, s)
            torch.cuda.synchronize()
            want = a + b if name.startswith("R2W1") else a
            assert torch.equal(c, want), name

    for rep in range(args.reps):
        for p in pats:
            for j in range(20):
                launch(p, j)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for j in range(steps):
                launch(p, j)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / steps
            tbs = p[2] * nbytes / us / 1e6
            print(json.dumps({"rep": rep, "lib": args.lib, "mib": args.mib, "pattern": p[0], "streams": p[2], "us": round(us, 2),
                              "TBs": round(tbs, 3), "frac_of_8TBs": round(tbs / 8.0, 4)}), flush=True)


if __name__ == "__main__":
    main()
