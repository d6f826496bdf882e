"""GPU: every surviving execution mode on a golden case of the reference
(the matrix: tests/mode_matrix.py).

One test per cell of route x signalling x launch mode x completion x arena:
the ranks run the cell's golden case three times (run 1 eager, run 2
captures where graphs apply, run 3 replays), every run equals the
reference's output byte for byte, and the executor reports the cell's mode.
Device signalling: ranks as processes on the box's GPU (each its own);
host signalling: ranks as threads of one process sharing the GPU.
tests/test_mode_matrix.py (CPU) fails if a cell has no case here.
"""
import json
import os
import subprocess
import sys
import tempfile
import threading
import uuid

import numpy as np
import pytest

import mode_matrix as mm

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RANK = os.path.join(ROOT, "tests", "mode_matrix_rank.py")


@pytest.fixture(scope="module")
def gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _run_processes(c, case, P):
    with tempfile.TemporaryDirectory() as d:
        env = dict(os.environ, **mm.env_of(c))
        procs = [subprocess.Popen([sys.executable, RANK, str(r), str(P), "file:" + os.path.join(d, "s"), case,
                                   c["completion"], c["arena"], os.path.join(d, f"o{r}.json")], env=env,
                                  stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(P)]
        errs = []
        try:
            for p in procs:
                errs.append(p.communicate(timeout=150)[1])
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        assert [p.returncode for p in procs] == [0] * P, "\n".join(e[-2000:] for e in errs)
        return [json.load(open(os.path.join(d, f"o{r}.json"))) for r in range(P)]


def _run_threads(c, case, P, monkeypatch):
    import mode_matrix_rank
    for k, v in mm.env_of(c).items():
        monkeypatch.setenv(k, v)
    url = "mem:" + uuid.uuid4().hex
    res, errors = [None] * P, []

    def body(r):
        try:
            res[r] = mode_matrix_rank.run_rank(r, P, url, case, c["completion"], c["arena"])
        except Exception as e:  # noqa: BLE001
            errors.append((r, repr(e)))

    ts = [threading.Thread(target=body, args=(r,)) for r in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(150)
    assert not errors, errors
    return res


@pytest.mark.timeout(200)
@pytest.mark.parametrize("cell", mm.cells(), ids=mm.cell_id)
def test_mode_cell_golden(gpu, golden_sched, cell, monkeypatch):
    case, _ = mm.CASES[cell["route"]]
    P = int(case.split("/")[3][1:])
    want = golden_sched[case + "/out"]
    res = (_run_processes(cell, case, P) if cell["signal"] == "device"
           else _run_threads(cell, case, P, monkeypatch))
    for r, x in enumerate(res):
        for it, hx in enumerate(x["outs"]):
            got = np.frombuffer(bytes.fromhex(hx), dtype=want.dtype)
            assert got.shape == want.shape and (got.view(np.uint8) == want.view(np.uint8)).all(), (r, it)
        mm.check_mode(cell, x["modes"])
