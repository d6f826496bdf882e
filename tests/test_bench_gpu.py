"""GPU: bench.py's multi-rank section as a regression test (2 ranks on the
box's GPU, relaunched by bench.py through torch.distributed.run).

The config-3 variants run back to back in the same rank processes, each on a
new context and algorithm.  Before the IPC slab pool (gloo_amd/ipc.h), a
ring-route executor created right after one that had REPLAYED A hipGraph
WITH MEMCPY NODES into the peer's same-size inbox imported the previous
inbox's pages: the graph kept the import alive past hipIpcCloseMemHandle,
and the peer's next arena came back at the same address with a byte-identical
handle (profiles/round3/r3g_ipc_bisect_no_pool.jsonl).  Exported slabs are
now never freed and imports never closed, so every variant must verify in
bench.py's order and in the order that provoked the stale import — no error
accepted, no retry in the library.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(variants, full=False):
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20", "--warmup", "5",
           "--config3-only"]
    if variants:
        cmd += ["--config3-variants", variants]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=380, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    x = out["xgmi_allreduce"]
    assert x.get("verified") is True, x
    assert x["variants"], x
    return out if full else x["variants"]


@pytest.fixture(scope="module")
def gpu():
    pytest.importorskip("torch")
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.timeout(400)
def test_config3_variants_in_bench_order_verified(gpu):
    out = run_bench("", full=True)
    for name, v in out["xgmi_allreduce"]["variants"].items():
        assert v.get("verified") is True, (name, v)
    # SURVEY 8(e) twice: the unfused mesh (a pure fold kernel, the
    # event-profiled runs) and the default schedule as it ships (fold +
    # forward fused, stamped as one)
    eff = out["per_gpu_efficiency"]
    assert eff["value"] and "unfused" in eff["data_path"], eff
    assert eff["fused_default"]["value"] and "fused" in eff["fused_default"]["data_path"], eff
    assert "fold + forward fused" in out["xgmi_allreduce"]["schedule"], out["xgmi_allreduce"]
    assert set(out["xgmi_allreduce"]["variants"]) == {"ring_graph", "ring_eager", "mesh_graph",
                                                      "mesh_host_workspace"}, out["xgmi_allreduce"]["variants"]
    assert out["xgmi_allreduce"]["section_s"]["config3"] > 0


@pytest.mark.timeout(200)
def test_watchdog_fire_exits_nonzero(gpu):
    """A hung N>1 section must show in the driver's record: the watchdog
    prints the line with the section marked timed out, then the job fails."""
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20", "--warmup", "5",
           "--config3-only", "--no-cpu", "--no-host-staged", "--watchdog-seconds", "0.5"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, cwd=ROOT)
    assert r.returncode != 0, r.stdout[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert "watchdog" in out["xgmi_allreduce"]["error"], out["xgmi_allreduce"]
    assert out["value"] > 0


@pytest.mark.timeout(400)
def test_config3_variants_in_provoking_order_verified(gpu):
    got = run_bench("ring_graph,ring_eager,mesh_graph,ring_eager")
    for name, v in got.items():
        assert v.get("verified") is True, (name, v)
