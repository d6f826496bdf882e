"""CPU: the schedule planners (plan.cc, mesh.cc — the host code that turns
the reference's algorithms into plans) under AddressSanitizer and
UndefinedBehaviorSanitizer.  SURVEY §5 lists the reference's -DSANITIZE
builds; GPU sanitizers are unavailable on this pool, so the host side is
checked here: a host-only build of the planners, loaded into a child Python
with libasan preloaded, plans every algorithm over a grid of sizes and runs
the all-rank simulation on a subset.
"""
import os
import shutil
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DRIVER = r'''
import os, sys
sys.path.insert(0, os.path.join(os.environ["GLOO_AMD_ROOT"], "tests"))
sys.path.insert(0, os.environ["GLOO_AMD_ROOT"])
import numpy as np
from plan_sim import get_plan, simulate
algos = ["ring_chunked", "halving_doubling", "ring", "local", "allreduce_new", "allreduce_bcube", "bcube",
         "mesh_ring_chunked", "mesh_halving_doubling", "mesh_allreduce_new", "mesh_allreduce_bcube"]
n_plans = 0
for P in (1, 2, 3, 5, 6, 8, 12):
    for n in (0, 1, 7, 1000, 4099):
        for algo in algos:
            if algo.startswith("mesh_") and not 2 <= P <= 8:
                continue
            if algo == "local" and P != 1:
                continue
            for r in range(P):
                get_plan(algo, r, P, n, 1, None, elem_size=4, max_seg=128)
                n_plans += 1
        recv = np.array([n // P + (1 if q < n % P else 0) for q in range(P)], np.int32)
        for r in range(P):
            get_plan("reduce_scatter", r, P, n, 1, recv)
            get_plan("reduce", r, P, n, 1, np.array([P - 1], np.int32), elem_size=8, max_seg=256)
            if 2 <= P <= 8:
                get_plan("mesh_reduce_scatter", r, P, n, 1, recv)
                get_plan("mesh_reduce", r, P, n, 1, np.array([0], np.int32), elem_size=8)
            n_plans += 4
x = np.random.default_rng(0).standard_normal((6, 1, 999)).astype(np.float32)
for algo in ("halving_doubling", "mesh_halving_doubling", "allreduce_bcube", "mesh_allreduce_bcube"):
    simulate(algo, "sum", "f32", x, seed=1)
simulate("mesh_reduce", "sum", "f32", x, recv=np.array([2], np.int32), seed=1)
for base in (2, 3, 1 << 30):
    simulate("bcube", "sum", "f32", x, recv=np.array([base], np.int32), seed=1)
print("planned", n_plans)
'''


def test_planners_under_asan_ubsan():
    gxx = shutil.which("g++") or shutil.which("gcc")
    if gxx is None:
        pytest.skip("no host compiler")
    libasan = subprocess.run([gxx, "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(libasan) or not os.path.exists(libasan):
        pytest.skip("libasan not available")
    with tempfile.TemporaryDirectory() as d:
        lib = os.path.join(d, "libplan_asan.so")
        cmd = [gxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
               "-fno-omit-frame-pointer", "-fPIC", "-shared", "-I" + os.path.join(ROOT, "include"),
               "-I" + os.path.join(ROOT, "gloo_amd", "include"), os.path.join(ROOT, "gloo_amd", "csrc", "plan.cc"),
               os.path.join(ROOT, "gloo_amd", "csrc", "mesh.cc"), "-o", lib]
        b = subprocess.run(cmd, capture_output=True, text=True)
        assert b.returncode == 0, b.stderr
        drv = os.path.join(d, "drv.py")
        open(drv, "w").write(DRIVER)
        env = dict(os.environ, GLOO_AMD_ROOT=ROOT, GLOO_AMD_PLAN_LIB=lib, LD_PRELOAD=libasan,
                   ASAN_OPTIONS="detect_leaks=0:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
        r = subprocess.run([sys.executable, drv], capture_output=True, text=True, env=env, timeout=900)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
        assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
        assert "planned" in r.stdout
