"""CPU: the execution-mode matrix and the knob list are closed.

  * every cell of route x signalling x launch x completion x arena that the
    executor can run (tests/mode_matrix.py) has a golden GPU case in
    tests/test_mode_matrix_gpu.py (checked on its collected ids), on a golden
    fixture that exists, and the sliced cells' cases do slice (plan_sim);
  * the environment variables the library reads (getenv in gloo_amd/csrc)
    are exactly the rows of INTEGRATION.md §4, and the matrix selects its
    cells with those alone.
"""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import mode_matrix as mm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cells_are_the_product_minus_the_structural_exclusions():
    cells = mm.cells()
    n = len(mm.ROUTES) * len(mm.SIGNALS) * len(mm.LAUNCHES) * len(mm.COMPLETIONS) * len(mm.ARENAS)
    excluded = [c for c in __import__("itertools").product(mm.ROUTES, mm.SIGNALS, mm.LAUNCHES, mm.COMPLETIONS,
                                                            mm.ARENAS) if not mm.possible(*c)]
    assert len(cells) + len(excluded) == n
    # host waits: eager only; HOST-workspace inboxes: never sliced
    for route, signal, launch, completion, arena in excluded:
        assert (signal == "host" and launch != "eager") or (arena == "host" and launch == "sliced")
    assert len(cells) == 36
    assert len({mm.cell_id(c) for c in cells}) == len(cells)


def test_every_cell_has_a_golden_gpu_case():
    z = np.load(os.path.join(ROOT, "tests", "golden", "sched_golden.npz"))
    for case, _ in mm.CASES.values():
        assert case + "/in" in z.files and case + "/out" in z.files, case
    out = subprocess.run([sys.executable, "-m", "pytest", "--collect-only", "-q", "-m", "gpu",
                          "tests/test_mode_matrix_gpu.py"], cwd=ROOT, capture_output=True, text=True, timeout=300)
    ids = {ln.split("[", 1)[1].rstrip("]") for ln in out.stdout.splitlines() if "test_mode_cell_golden[" in ln}
    assert ids == {mm.cell_id(c) for c in mm.cells()}, (sorted(ids), out.stderr[-2000:])


@pytest.mark.parametrize("route", mm.ROUTES)
def test_sliced_cells_slice(route):
    """The sliced cells' case, route and slice bytes give more than one slice
    on every rank (the rule of executor.cc proposeSlices, restated in
    plan_sim.sliceable), so the GPU assertion tests the sliced interpreter."""
    from plan_sim import get_plan, sliceable
    case, sb = mm.CASES[route]
    algo, P, n = case.split("/")[0], int(case.split("/")[3][1:]), int(case.split("/")[-1][1:])
    plan = {"mesh": {"ring_chunked": "ring_chunked_mesh", "halving_doubling": "mesh_halving_doubling"},
            "reference": {"ring_chunked": "ring_chunked_pipe", "halving_doubling": "halving_doubling"}}[route][algo]
    for r in range(P):
        steps, _ = get_plan(plan, r, P, n, 1, None, elem_size=4)
        biggest = max(s.length for s in steps) * 4
        assert sliceable(plan, P, n, r, elem_size=4), (case, route, r)
        assert -(-biggest // int(sb)) > 1 and biggest <= 32 * 2 * int(sb), (case, route, r, biggest)


def _knobs_read():
    names = set()
    for f in os.listdir(os.path.join(ROOT, "gloo_amd", "csrc")):
        text = open(os.path.join(ROOT, "gloo_amd", "csrc", f)).read()
        names |= set(re.findall(r'getenv\("(GLOO_AMD_[A-Z0-9_]+)"\)', text))
    return names


def _knobs_documented():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text.split("## 4.", 1)[1].split("\n## ", 1)[0].split("Removed in round 6", 1)[0]
    return set(re.findall(r"^\| `(GLOO_AMD_[A-Z0-9_]+)`", sec, re.M))


def test_integration_lists_exactly_the_knobs_the_library_reads():
    assert _knobs_read() == _knobs_documented(), (sorted(_knobs_read()), sorted(_knobs_documented()))


def test_matrix_selects_cells_with_surviving_knobs_only():
    read = _knobs_read()
    for c in mm.cells():
        assert set(mm.env_of(c)) <= read, c
