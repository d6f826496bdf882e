"""CPU: no stray files in the tree (a '--help' file created by
a tool run was committed twice)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_no_file_named_like_a_flag():
    strays = [f for f in os.listdir(ROOT) if f.startswith("-")]
    assert not strays, strays
    try:
        out = subprocess.run(["git", "ls-files"], cwd=ROOT, capture_output=True, text=True, timeout=60)
    except (OSError, subprocess.TimeoutExpired):
        pytest.skip("git not available")
    if out.returncode != 0:
        pytest.skip("not a git checkout")
    tracked = [f for f in out.stdout.splitlines() if os.path.basename(f).startswith("-")]
    assert not tracked, tracked


def test_gpu_run_starts_with_hot_path_parity():
    """under `pytest -m gpu -x` the kernel's own parity suite
    (tests/test_reduce_gpu.py, config 2's 64 MiB case first) is collected
    before any collective file, so a collective failure cannot leave it
    unrun."""
    import sys
    out = subprocess.run([sys.executable, "-m", "pytest", "--collect-only", "-q", "-m", "gpu", "tests"],
                         cwd=ROOT, capture_output=True, text=True, timeout=600)
    ids = [ln for ln in out.stdout.splitlines() if "::" in ln]
    assert ids, out.stdout[-2000:] + out.stderr[-2000:]
    assert ids[0] == "tests/test_reduce_gpu.py::test_full_size_64mib_f32_sum_properties", ids[:3]
    files = [i.split("::")[0] for i in ids]
    k = files.count("tests/test_reduce_gpu.py")
    assert k > 50 and files[:k] == ["tests/test_reduce_gpu.py"] * k, files[:k + 1]
    for name in ("test_golden_reduce3", "test_golden_nan_payloads", "test_misaligned_offsets",
                 "test_beyond_4gi_elements"):
        assert any(name in i for i in ids[:k]), name


def test_no_hipipc_in_the_product():
    """cross-process device memory goes through dma-bufs (VMM
    slabs, exported ranges of a caller's allocation), never hipIpc handles."""
    hits = []
    for base in ("gloo_amd/csrc", "gloo_amd/include", "include"):
        for dirpath, _, files in os.walk(os.path.join(ROOT, base)):
            for f in files:
                text = open(os.path.join(dirpath, f), errors="replace").read()
                for name in ("hipIpcGetMemHandle", "hipIpcOpenMemHandle", "hipIpcCloseMemHandle"):
                    if name in text:
                        hits.append((os.path.join(dirpath, f), name))
    assert not hits, hits
