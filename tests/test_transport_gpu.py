"""GPU: the xGMI transport with Gloo's transport::Pair / Buffer shape
(gloo_amd/include/gloo_amd/transport.h).  examples/transport_ring_chunked
runs gloo::AllreduceRingChunked's run() (gloo/allreduce_ring_chunked.h:83-212)
statement for statement over it — createSendBuffer / createRecvBuffer with
the reference's slots, Buffer::send(offset, length), waitRecv, the
notification handshake, the 1-element dummy send for empty chunks — on
device buffers, with the per-chunk reduction done by the HIP kernel; every
element checked against a closed form, over several runs."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "transport_ring_chunked")


@pytest.mark.timeout(300)
@pytest.mark.parametrize("P,count,runs", [(2, 1000, 3), (3, 100003, 2), (4, 1 << 22, 2), (8, 1 << 20, 2),
                                          (5, 7, 2), (1, 4099, 1)])
def test_transport_ring_chunked(P, count, runs):
    pytest.importorskip("torch")
    if not os.path.exists(EXE):
        pytest.skip("example not built")
    r = subprocess.run([EXE, str(P), str(count), str(runs)], capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok"), r.stdout


@pytest.mark.timeout(300)
@pytest.mark.parametrize("P,count", [(2, 100003), (4, 1 << 20)])
def test_transport_ring_chunked_processes(tmp_path, P, count):
    """The same with ranks as processes: receive buffers exported as HIP IPC
    handles through a file store, arrivals through the node's control block."""
    pytest.importorskip("torch")
    if not os.path.exists(EXE):
        pytest.skip("example not built")
    procs = [subprocess.Popen([EXE, str(P), str(count), "2", str(r), str(tmp_path / "store")],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(P)]
    outs = [p.communicate(timeout=280)[0] for p in procs]
    assert [p.returncode for p in procs] == [0] * P, outs
    assert all(o.startswith("ok") for o in outs), outs
