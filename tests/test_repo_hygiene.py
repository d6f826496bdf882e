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
