"""CPU: the C-ABI library loads, exports every symbol include/gloo_amd.h
declares, and rejects bad arguments without touching the GPU."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    text = open(os.path.join(ROOT, "include", "gloo_amd.h")).read()
    return sorted(set(re.findall(r"^\s*[\w\s\*]+?\b(gloo_hip_\w+)\s*\(", text, re.M)))


def test_header_declares_expected_entry_points():
    import gloo_amd
    assert set(declared_functions()) == set(gloo_amd.EXPORTED)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(os.path.join(ROOT, "gloo_amd", "libgloo_amd.so"))
    for name in declared_functions():
        assert hasattr(lib, name), name


def test_zero_length_and_argument_errors():
    import gloo_amd
    # n == 0 is a no-op that never reaches HIP (gloo allows count == 0)
    assert gloo_amd.lib.gloo_hip_reduce(1, 8, None, None, 0, None) == 0
    assert gloo_amd.lib.gloo_hip_reduce3(3, 6, None, None, None, 0, None) == 0
    assert gloo_amd.lib.gloo_hip_reduce(7, 8, None, None, 0, None) == -1
    assert b"op" in gloo_amd.lib.gloo_hip_last_error()
    assert gloo_amd.lib.gloo_hip_reduce(1, 42, None, None, 0, None) == -2
    assert gloo_amd.lib.gloo_hip_reduce(1, 8, None, None, 5, None) == -3
    arr = (ctypes.c_void_p * 1)(None)
    assert gloo_amd.lib.gloo_hip_reduce_multi(1, 8, None, arr, 0, 5, None) == -4
    assert gloo_amd.lib.gloo_hip_reduce_multi(1, 8, None, arr, 9, 5, None) == -4
    with pytest.raises(gloo_amd.GlooHipError):
        gloo_amd.reduce_ptr("sum", "f32", 0, 0, 5)


def test_dtype_sizes():
    import gloo_amd
    want = {"i8": 1, "u8": 1, "i32": 4, "u32": 4, "i64": 8, "u64": 8, "f16": 2, "bf16": 2,
            "f32": 4, "f64": 8}
    for k, v in want.items():
        assert gloo_amd.dtype_size(k) == v
    assert gloo_amd.dtype_size(99) == 0


def test_op_and_dtype_codes_mirror_reference():
    """gloo::ReductionType values (gloo/algorithm.h:49-57)."""
    import gloo_amd
    import oracle
    assert [int(gloo_amd.ReductionType[x]) for x in ("SUM", "PRODUCT", "MAX", "MIN")] == [1, 2, 3, 4]
    for name, (code, _) in oracle.DTYPES.items():
        assert int(gloo_amd.DTYPE_NAMES[name]) == code


def test_set_profiling_modes_reach_the_c_abi(monkeypatch):
    """Algorithm.set_profiling passes 0 / 1 (events) / 2 (device stamps)
    through unchanged; True stays the event mode."""
    import gloo_amd
    seen = []

    def fake(h, mode):
        seen.append(mode)
        return 0
    monkeypatch.setattr(gloo_amd.lib, "gloo_hip_algorithm_set_profiling", fake)
    a = gloo_amd.Algorithm.__new__(gloo_amd.Algorithm)
    a._h = None
    for on in (True, False, 0, 1, 2):
        a.set_profiling(on)
    assert seen == [1, 0, 0, 1, 2]


def test_library_built_from_this_tree():
    """gloo_hip_version() carries a hash of the sources the library was built
    from (gloo_amd/srchash.py); it must be this tree's, so no stale prebuilt
    .so can stand in for the sources (smoke() checks the same on the GPU)."""
    import gloo_amd
    from gloo_amd import srchash
    assert gloo_amd.version() == srchash.version_string()


def test_source_hash_covers_every_library_source():
    from gloo_amd import srchash
    _, files = srchash.source_files()
    src = os.path.join(ROOT, "gloo_amd", "csrc")
    for f in os.listdir(src):
        assert os.path.join("gloo_amd", "csrc", f) in files, f
    assert os.path.join("include", "gloo_amd.h") in files
