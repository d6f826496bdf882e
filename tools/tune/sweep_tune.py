"""TUNING ONLY: time every variant of tools/tune/libtune.so on a 64 MiB
fp32 in-place sum with 6 rotated pairs; checks each variant's result."""
import ctypes, json, os, sys
import torch
L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libtune.so"))
L.tune_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
n = 16 << 20
pairs = [(torch.rand(n, device="cuda"), torch.rand(n, device="cuda")) for _ in range(6)]
chk_a, chk_b = torch.rand(n, device="cuda"), torch.rand(n, device="cuda")
s = torch.cuda.current_stream().cuda_stream
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
res = []
for rep in range(2):
    for i in range(L.tune_count()):
        d = (ctypes.c_int * 6)(); L.tune_desc(i, d)
        c = torch.empty_like(chk_a)
        L.tune_run(i, c.data_ptr(), chk_a.data_ptr(), chk_b.data_ptr(), n, s)
        ok = bool(torch.equal(c, chk_a + chk_b))
        for j in range(20):
            x, y = pairs[j % 6]; L.tune_run(i, x.data_ptr(), x.data_ptr(), y.data_ptr(), n, s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(); e0.record()
        for j in range(steps):
            x, y = pairs[j % 6]; L.tune_run(i, x.data_ptr(), x.data_ptr(), y.data_ptr(), n, s)
        e1.record(); torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / steps
        r = {"rep": rep, "i": i, "unroll": d[0], "laux": d[1], "saux": d[2], "block": d[3], "grid": d[4], "xcd": d[5],
             "us": round(us, 2), "TBs": round(3 * n * 4 / us / 1e6, 3), "ok": ok}
        print(json.dumps(r), flush=True)
