"""GPU: AllreduceBcube / CudaAllreduceBcube (gloo/allreduce_bcube.h,
gloo/cuda_allreduce_bcube.{h,cc}) through the HIP plan executor, byte for
byte against the reference's own outputs (tests/golden/bcube_golden.npz,
every rank's).  Ranks as threads of one process for every golden case; ranks
as processes (tests/sched_pool.py batches) for a subset, in the default
launch modes, with graph replay forced, with the interpreter off and on the
reference route.  For 2 <= P <= 8 the default is the derived mesh plan
wherever it exists (gloo_amd/csrc/mesh.cc; tests/test_bcube_plan.py lists
which cases), else the reference route.  The base rides in recv_elems[0]
(gloo::Context::base, gloo/context.h:28-33)."""
import os

import numpy as np
import pytest

import sched_pool
from test_collectives_gpu import run_threads, same_bytes

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "bcube_golden.npz")


@pytest.fixture(scope="module")
def torch():
    t = pytest.importorskip("torch")
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.fixture(scope="module")
def golden():
    return np.load(GOLDEN)


def _keys():
    z = np.load(GOLDEN)
    return sorted({k.rsplit("/", 1)[0] for k in z.files})


def _base(case):
    return int(case.split("/")[4][1:])


@pytest.mark.parametrize("case", _keys())
def test_bcube_threads_golden(torch, golden, case):
    op, dtype = case.split("/")[1:3]
    x, want = golden[case + "/in"], golden[case + "/out"]
    y = run_threads(torch, "bcube", op, dtype, x, recv=[_base(case)])
    for r in range(y.shape[0]):
        for j in range(y.shape[1]):
            assert same_bytes(y[r, j], want[r]), (r, j)


@pytest.mark.parametrize("case", ["bcube/sum/f32/P8/b2/k1/n1000", "bcube/sum/f32/P4/b4/k1/n64",
                                  "bcube/sum/f32/P4/b2/k3/n1000", "bcube/max/f32/P8/b2/k1/n4099"])
def test_bcube_threads_reference_route(torch, golden, case, monkeypatch):
    """The reference's own route (GLOO_AMD_MESH=0) where the default is the
    derived mesh plan (2 <= P <= 8 with a mesh form)."""
    monkeypatch.setenv("GLOO_AMD_MESH", "0")
    op, dtype = case.split("/")[1:3]
    x, want = golden[case + "/in"], golden[case + "/out"]
    y = run_threads(torch, "bcube", op, dtype, x, recv=[_base(case)])
    for r in range(y.shape[0]):
        for j in range(y.shape[1]):
            assert same_bytes(y[r, j], want[r]), (r, j)


@pytest.mark.parametrize("P,base", [(8, 2), (9, 3), (16, 4)])
def test_bcube_threads_repeated_runs_and_user_stream(torch, P, base):
    """Closed form of gloo/test/base_test.h:184-236 (input j*P + rank): one run
    on a caller's stream, then three runs of max on the algorithm's own stream."""
    n = 4099
    x = np.array([[np.arange(n, dtype=np.float32) * P + r] for r in range(P)], dtype=np.float32)
    y = run_threads(torch, "bcube", "sum", "f32", x, recv=[base], stream=True)
    want = np.arange(n, dtype=np.float64) * P * P + P * (P - 1) / 2
    assert (y[:, 0] == want.astype(np.float32)).all()
    y3 = run_threads(torch, "bcube", "max", "f32", x, recv=[base], runs=3)
    assert (y3[:, 0] == (np.arange(n) * P + P - 1).astype(np.float32)).all()


PROCESS_CASES = [
    ("bcube/sum/f32/P8/b2/k1/n1000", {}, 1),
    ("bcube/sum/f32/P8/b2/k1/n20011", {}, 1),
    ("bcube/sum/bf16/P8/b2/k1/n2000", {}, 1),
    ("bcube/sum/f32/P9/b3/k1/n4099", {}, 1),
    ("bcube/sum/f32/P4/b4/k1/n1000", {}, 1),
    ("bcube/max/f32/P8/b2/k1/n4099", {"GLOO_AMD_GRAPH": "1"}, 3),
    ("bcube/sum/f32/P4/b2/k1/n1000", {"GLOO_AMD_INTERP": "0"}, 3),
    ("bcube/sum/f32/P8/b2/k1/n20011", {"GLOO_AMD_MESH": "0"}, 1),
    ("bcube/sum/f32/P4/b4/k1/n1000", {"GLOO_AMD_MESH": "0"}, 1),
]
for _c, _e, _n in PROCESS_CASES:
    sched_pool.register(_c, _e, _n)


@pytest.mark.parametrize("case,env,runs", PROCESS_CASES)
def test_bcube_processes_golden(torch, golden, case, env, runs):
    """Every run of every rank process equals that rank's reference output
    (each run starts from the case's input)."""
    res = sched_pool.result(case, env, runs)
    assert res.err is None, res.err
    want = golden[case + "/out"]
    for it in range(runs):
        for r in range(len(res.outs)):
            assert same_bytes(res.outs[r][it], want[r]), (r, it)
    if env.get("GLOO_AMD_INTERP") == "0":
        assert not any(m["interp"] for ms in res.modes for m in ms), res.modes
