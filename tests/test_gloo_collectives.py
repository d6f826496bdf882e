"""gloo::hip::allreduce / gloo::hip::reduce (gloo_amd/include/gloo_amd/gloo_collectives.h):
the reference's own gloo::AllreduceOptions / gloo::ReduceOptions, filled with
device pointers and the reference's gloo::sum/product/max/min<T> as a Gloo
program fills them for gloo::allreduce / gloo::reduce, run on the MI355X
path.  oracle/_ref/newstyle_test is that Gloo program (built against the
reference's headers and objects; ranks are threads over its TCP transport).

Expected bytes: the reference's own outputs for the same inputs —
tests/golden/sched_golden.npz (allreduce_new/: the RING algorithm) and
tests/golden/newstyle_golden.npz (bcube/, reduce/), from oracle/gen_golden.py.
Every rank calls twice; both calls must match.  For reduce on the device
path only the root's output is defined (the default mesh route leaves other
scratch on the other ranks); over the hip transport the reference's own
algorithm runs, so every rank's output matches.

CPU: the header is Gloo-side only and the program exists when the reference
was available at build time.
"""
import os
import subprocess
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROGRAM = os.path.join(ROOT, "oracle", "_ref", "newstyle_test")
SCHED = os.path.join(ROOT, "tests", "golden", "sched_golden.npz")
NEWSTYLE = os.path.join(ROOT, "tests", "golden", "newstyle_golden.npz")


def _cases():
    out = []
    z = np.load(SCHED)
    out += [("sched", k) for k in sorted({k.rsplit("/", 1)[0] for k in z.files if k.startswith("allreduce_new/")})]
    z = np.load(NEWSTYLE)
    out += [("newstyle", k) for k in sorted({k.rsplit("/", 1)[0] for k in z.files})]
    # thread ranks of one process share the GPU: keep P small enough to stay quick
    return [c for c in out if int(c[1].split("/")[3][1:]) <= 8]


def test_header_is_gloo_side_only():
    text = open(os.path.join(ROOT, "gloo_amd", "include", "gloo_amd", "gloo_collectives.h")).read()
    assert '#include "gloo/allreduce.h"' in text and '#include "gloo/reduce.h"' in text
    for f in os.listdir(os.path.join(ROOT, "gloo_amd", "csrc")):
        assert "gloo_collectives.h" not in open(os.path.join(ROOT, "gloo_amd", "csrc", f)).read(), f


def _meta(src, case):
    z = np.load(SCHED if src == "sched" else NEWSTYLE)
    parts = case.split("/")
    kind = {"allreduce_new": "ring", "bcube": "bcube", "reduce": "reduce"}[parts[0]]
    op, dtype, P = parts[1], parts[2], int(parts[3][1:])
    if kind == "reduce":
        nin, n, root, seg = int(parts[4][1:]), int(parts[5][1:]), int(parts[6][1:]), int(parts[7][1:])
        nout = 1
    else:
        nin, nout, n, seg = int(parts[4][1:]), int(parts[5][1:]), int(parts[6][1:]), int(parts[7][1:])
        root = 0
    return z, kind, op, dtype, P, nin, nout, n, root, seg


_batches = {}  # mode -> (tempdir, {(src, case): case dir})


def _batch(mode):
    """Every case of `mode` in ONE run of the program (newstyle_test --batch):
    a process per case cost more than the cases themselves."""
    if mode not in _batches:
        root = tempfile.mkdtemp(prefix="gloo_opts_")
        dirs = {}
        for i, (src, case) in enumerate(_cases()):
            z, kind, op, dtype, P, nin, nout, n, rt, seg = _meta(src, case)
            d = os.path.join(root, f"c{i}")
            os.makedirs(d)
            open(os.path.join(d, "meta.txt"), "w").write(f"{kind} {op} {dtype} {P} {nin} {nout} {n} {rt} {seg}\n")
            z[case + "/init"].tofile(os.path.join(d, "init.bin"))
            if nin:
                z[case + "/in"].tofile(os.path.join(d, "in.bin"))
            dirs[(src, case)] = d
        lst = os.path.join(root, "list.txt")
        open(lst, "w").write("\n".join(dirs.values()) + "\n")
        r = subprocess.run([PROGRAM, "--batch", lst, mode], capture_output=True, text=True, timeout=600)
        _batches[mode] = (root, dirs, r.stdout[-3000:] + r.stderr[-3000:])
    return _batches[mode]


@pytest.fixture(scope="module", autouse=True)
def _cleanup_batches():
    yield
    import shutil
    for root, _, _ in _batches.values():
        shutil.rmtree(root, ignore_errors=True)
    _batches.clear()


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", ["device", "hip-transport-host"])
@pytest.mark.parametrize("src,case", _cases())
def test_gloo_options_golden(src, case, mode):
    """mode device: gloo::hip::allreduce / reduce on device buffers (the
    MI355X path).  mode hip-transport-host: the reference's own
    gloo::allreduce / gloo::reduce on host buffers, unchanged, over a
    gloo::Context whose pairs are the hip transport (its unbound buffers)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(PROGRAM):
        pytest.skip("oracle/_ref/newstyle_test not built (needs /root/reference at build time)")
    z, kind, op, dtype, P, nin, nout, n, root, seg = _meta(src, case)
    init = z[case + "/init"]
    want = z[case + "/out"]
    _, dirs, log = _batch(mode)
    d = dirs[(src, case)]
    res = os.path.join(d, "result.txt")
    assert os.path.exists(res), "the batch ended before this case: " + log
    text = open(res).read()
    assert text.startswith("ok"), text
    for rank in range(P):
        if kind == "reduce" and rank != root and mode == "device":
            continue  # the mesh route leaves other scratch there (the reference's algorithm: partials)
        for call in range(2):
            got = np.fromfile(os.path.join(d, f"out_{rank}_{call}.bin"), dtype=init.dtype).reshape(nout, n)
            expect = want[rank] if kind == "reduce" else want
            for j in range(nout):
                assert got[j].view(np.uint8).tobytes() == expect.view(np.uint8).tobytes(), (rank, call, j)
