"""CPU: the GPU suite keeps every golden family (VERDICT r4 "next round" 3).

Collects the `-m gpu` set (collection only, no GPU needed) and checks that
every case of every committed golden file (tests/golden/*.npz: the
reference's own outputs, oracle/gen_golden.py) is named by at least one GPU
test id, so trimming the suite for time cannot silently drop one."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def gpu_ids():
    r = subprocess.run([sys.executable, "-m", "pytest", "tests", "-m", "gpu", "--collect-only", "-q",
                        "-p", "no:cacheprovider"], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    ids = [ln for ln in r.stdout.splitlines() if "::" in ln]
    assert len(ids) > 500, r.stdout[-2000:]
    return "\n".join(ids)


def cases(name):
    z = np.load(os.path.join(GOLDEN, name))
    return sorted({k.rsplit("/", 1)[0] for k in z.files})


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", ["sched_golden.npz", "newstyle_golden.npz", "math_golden.npz",
                                  "bw_golden.npz", "bcube_golden.npz"])
def test_every_golden_case_has_a_gpu_test(gpu_ids, name):
    cs = cases(name)
    assert cs
    missing = [c for c in cs if c not in gpu_ids]
    assert not missing, f"{name}: {len(missing)} golden cases no GPU test names: {missing[:10]}"


@pytest.mark.timeout(600)
def test_gpu_extended_cases_leave_the_default_run():
    """gpu_extended variants (conftest.py) are deselected from `-m gpu` unless
    GLOO_AMD_GPU_EXTENDED=1, and nothing else is."""
    def collect(extra):
        env = dict(os.environ, **extra)
        env.pop("GLOO_AMD_GPU_EXTENDED", None) if not extra else None
        r = subprocess.run([sys.executable, "-m", "pytest", "tests", "-m", "gpu", "--collect-only", "-q",
                            "-p", "no:cacheprovider"], cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        return {ln for ln in r.stdout.splitlines() if "::" in ln}
    default, extended = collect({}), collect({"GLOO_AMD_GPU_EXTENDED": "1"})
    assert default < extended
    extra = extended - default
    assert extra and all("test_ipc_arena_of_2gib_and_more" in t for t in extra), sorted(extra)
