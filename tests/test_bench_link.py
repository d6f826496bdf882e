"""CPU: the xGMI link bounds bench.py reports for config 3 (bench.link_bounds)
and the shape of its link figures: the bounds come from
the figure measured with the engine and pattern the route uses, name it, and
are null with the reason when it could not be measured (one GPU)."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_bounds_from_the_named_figures(bench):
    P, S, t = 8, 256 << 20, 0.010
    figs = {k: {"GBps": None, "why": "x"} for k in bench.LINK_FIGURES}
    figs[bench.RING_BOUND_FIGURE] = {"GBps": 50.0}
    figs[bench.MESH_BOUND_FIGURE] = {"peers": 7, "GBps_per_link": 40.0, "GBps_total": 280.0}
    b = bench.link_bounds(P, S, t, figs)
    ring_s = 2 * (P - 1) / P * S / 50e9
    mesh_s = 2 * S / P / 40e9
    assert b["ring_link_bound_ms"] == round(ring_s * 1e3, 3)
    assert b["mesh_link_bound_ms"] == round(mesh_s * 1e3, 3)
    assert b["frac_of_mesh_link_bound"] == round(mesh_s / t, 4)
    assert b["frac_of_ring_link_bound"] == round(ring_s / t, 4)
    assert b["busbw_frac_of_link"] == round(2 * (P - 1) / P * S / t / 50e9, 4)
    assert b["mesh_bound_figure"] == "kernel64_all_peers_one_gpu"
    assert b["ring_bound_figure"] == "kernel64_one_peer_one_dir"


def test_the_mesh_bound_uses_the_per_link_rate_not_the_total(bench):
    figs = {bench.RING_BOUND_FIGURE: {"GBps": 50.0},
            bench.MESH_BOUND_FIGURE: {"peers": 7, "GBps_per_link": 10.0, "GBps_total": 70.0}}
    b = bench.link_bounds(8, 8 << 20, 1.0, figs)
    assert b["mesh_link_bound_ms"] == round(2 * (8 << 20) / 8 / 10e9 * 1e3, 3)


def test_one_gpu_gives_null_bounds_with_the_reason(bench):
    why = "2 ranks on 1 GPU(s): no xGMI link to measure"
    figs = {k: {"GBps": None, "why": why} for k in bench.LINK_FIGURES}
    b = bench.link_bounds(2, 1 << 20, 0.001, figs)
    for route in ("ring", "mesh"):
        assert b[route + "_link_bound_ms"] is None
        assert b["frac_of_%s_link_bound" % route] is None
        assert b[route + "_bound_why"] == why
    assert b["busbw_frac_of_link"] is None


def test_link_figures_structure_without_a_second_gpu(bench):
    """The one-GPU rehearsal's structure (no torch.distributed needed)."""
    class FakeCuda:
        @staticmethod
        def device_count():
            return 1

    class FakeTorch:
        cuda = FakeCuda

    class FakeDist:
        @staticmethod
        def barrier():
            pass

        @staticmethod
        def broadcast_object_list(obj, src=0):
            pass

    link = bench.link_figures(FakeTorch, FakeDist, 0, 2, 1 << 20)
    assert set(link["figures"]) == set(bench.LINK_FIGURES)
    assert all(f["GBps"] is None and "no xGMI link" in f["why"] for f in link["figures"].values())
    assert link["mesh_bound_figure"] in link["figures"] and link["ring_bound_figure"] in link["figures"]


def test_config1_keeps_the_references_stdout_chatter_off_stdout(bench):
    """The reference's TCP context prints "[Gloo] Rank … connected" with
    std::cout (gloo/transport/tcp/context.cc:243-246); in round 6 those lines
    preceded the bench's JSON line on stdout.  config1 now sends fd 1 to
    stderr for the call: a child running it prints only its own line."""
    import subprocess
    import sys
    sys.path.insert(0, ROOT)
    import oracle
    if not oracle.ref_available():
        pytest.skip("oracle/_ref not built")
    code = ("import sys, types, json; sys.path.insert(0, %r); import bench, oracle; "
            "r = bench.config1(oracle, types.SimpleNamespace(config1_seconds=0.05), n=1 << 12); "
            "print(json.dumps(r))" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.startswith('{"elements": 4096'), r.stdout
    assert len(r.stdout.splitlines()) == 1, r.stdout
    assert "[Gloo] Rank" in r.stderr
