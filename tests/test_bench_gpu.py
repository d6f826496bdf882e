"""GPU: bench.py's multi-rank section as a regression test (2 ranks on the
box's GPU, relaunched by bench.py through torch.distributed.run).

The config-3 variants run back to back in the same rank processes, each on a
new context and algorithm.  A ring-route executor created right after one
whose sends were hipMemcpyAsync copies into the peer's same-size inbox was
seen to import the PREVIOUS inbox (its final contents showed through the new
mapping), and before the arena nonce check every message of that variant
went there while the arrival signals still came through.

bench.py's own order must give every variant `verified` (run 1 bit-exact
against the reference ring fold at 4096 sampled positions on every rank,
equal digests after the last run).  The order that provokes the stale import
must give, for every variant, either `verified` or the executor's explicit
refusal of the mapping — never a silently wrong result.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(variants):
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20", "--warmup", "5",
           "--config3-only"]
    if variants:
        cmd += ["--config3-variants", variants]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=380, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    x = json.loads(line)["xgmi_allreduce"]
    assert x.get("verified") is True, x
    assert x["variants"], x
    return x["variants"]


@pytest.fixture(scope="module")
def gpu():
    pytest.importorskip("torch")
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.timeout(400)
def test_config3_variants_in_bench_order_verified(gpu):
    for name, v in run_bench("").items():
        assert v.get("verified") is True, (name, v)


@pytest.mark.timeout(400)
def test_stale_import_refused_never_misdelivered(gpu):
    for name, v in run_bench("ring_memcpy,ring_kernel,mesh_memcpy_forked,ring_kernel").items():
        if v.get("verified") is True:
            continue
        assert "does not show its contents" in v.get("error", ""), (name, v)

