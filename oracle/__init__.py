"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by gloo_amd/.

Python loaders for the CPU checkers:
  * oracle/libgloo_oracle.so      the plain-C restatement of gloo/math.h
                                  (oracle/cpu_reduce.c), always available;
  * oracle/_ref/libgloo_ref.so    the reference itself compiled from
                                  /root/reference (oracle/Makefile); present in
                                  this container and travels to the GPU box as
                                  a built artefact, absent if never built;
  * oracle/schedules.py           numpy restatements of the reference's
                                  allreduce / reduce-scatter schedules.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

# dtype codes of include/gloo_amd.h <-> numpy storage dtypes (16-bit floats
# are carried as raw uint16 bits).
DTYPES = {
    "i8": (0, np.int8), "u8": (1, np.uint8), "i32": (2, np.int32), "u32": (3, np.uint32),
    "i64": (4, np.int64), "u64": (5, np.uint64), "f16": (6, np.uint16), "bf16": (7, np.uint16),
    "f32": (8, np.float32), "f64": (9, np.float64),
}
OPS = {"sum": 1, "product": 2, "max": 3, "min": 4}

_lib = None
_ref = None
_ref_base = None


def lib():
    """The plain-C oracle (oracle/cpu_reduce.c)."""
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "libgloo_oracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle not built: run `make -C oracle oracle`")
        L = ctypes.CDLL(path)
        L.oracle_reduce3.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_reduce_multi.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                          ctypes.c_size_t]
        L.oracle_f32_to_f16.argtypes = [ctypes.c_float]
        L.oracle_f32_to_f16.restype = ctypes.c_uint16
        L.oracle_f32_to_bf16.argtypes = [ctypes.c_float]
        L.oracle_f32_to_bf16.restype = ctypes.c_uint16
        L.oracle_sum_f32_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_size_t, ctypes.c_int]
        _lib = L
    return _lib


def ref_available():
    return os.path.exists(os.path.join(HERE, "_ref", "libgloo_ref.so"))


def ref():
    """The reference compiled from /root/reference (oracle/_ref/libgloo_ref.so)."""
    global _ref
    if _ref is None:
        L = ctypes.CDLL(os.path.join(HERE, "_ref", "libgloo_ref.so"))
        L.ref_reduce3.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_size_t]
        L.ref_reduce3_f16_scalar.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_size_t]
        L.ref_allreduce.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p,
                                    ctypes.c_void_p]
        L.ref_reduce_scatter.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p]
        L.ref_allreduce_new.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t,
                                        ctypes.c_void_p, ctypes.c_void_p]
        L.ref_allreduce_new_algo.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t,
                                             ctypes.c_void_p, ctypes.c_void_p]
        L.ref_allreduce_bcube.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
        L.ref_reduce_new.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                     ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.ref_allreduce_timed.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_double)]
        L.ref_allreduce_samples.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                            ctypes.c_double, ctypes.POINTER(ctypes.c_double), ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_int)]
        L.ref_last_error.restype = ctypes.c_char_p
        _ref = L
    return _ref


def ref_baseline():
    """gloo::sum<float> built as the reference ships it (oracle/ref_baseline.cc)."""
    global _ref_base
    if _ref_base is None:
        L = ctypes.CDLL(os.path.join(HERE, "_ref", "libgloo_ref_baseline.so"))
        L.ref_base_sum_f32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_size_t, ctypes.c_int]
        L.ref_base_sum2_f32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _ref_base = L
    return _ref_base


def reduce3(op, dtype, a, b):
    """c = a (op) b with the C oracle.  a, b: numpy arrays of the storage dtype."""
    code, npt = DTYPES[dtype]
    a = np.ascontiguousarray(a, dtype=npt)
    b = np.ascontiguousarray(b, dtype=npt)
    c = np.empty_like(a)
    rc = lib().oracle_reduce3(OPS[op], code, c.ctypes.data, a.ctypes.data, b.ctypes.data, a.size)
    if rc:
        raise RuntimeError(f"oracle_reduce3 failed: {rc}")
    return c


def reduce_multi(op, dtype, srcs):
    code, npt = DTYPES[dtype]
    srcs = [np.ascontiguousarray(s, dtype=npt) for s in srcs]
    dst = np.empty_like(srcs[0])
    arr = (ctypes.c_void_p * len(srcs))(*[s.ctypes.data for s in srcs])
    rc = lib().oracle_reduce_multi(OPS[op], code, dst.ctypes.data, arr, len(srcs), dst.size)
    if rc:
        raise RuntimeError(f"oracle_reduce_multi failed: {rc}")
    return dst


def ref_reduce3(op, dtype, a, b):
    """c = a (op) b computed by the reference's own gloo/math.h templates."""
    code, npt = DTYPES[dtype]
    a = np.ascontiguousarray(a, dtype=npt)
    b = np.ascontiguousarray(b, dtype=npt)
    c = np.empty_like(a)
    rc = ref().ref_reduce3(OPS[op], code, c.ctypes.data, a.ctypes.data, b.ctypes.data, a.size)
    if rc:
        raise RuntimeError(f"ref_reduce3 failed: {rc}")
    return c
