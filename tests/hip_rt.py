"""The few HIP runtime calls a test worker process needs (device memory and
copies), through ctypes on libamdhip64 — so a rank process starts in a
fraction of a second instead of importing torch.  Test infrastructure."""
import ctypes
import os

_lib = None


def lib():
    global _lib
    if _lib is None:
        for name in ("libamdhip64.so", os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib",
                                                      "libamdhip64.so")):
            try:
                _lib = ctypes.CDLL(name)
                break
            except OSError:
                continue
        if _lib is None:
            raise OSError("libamdhip64.so not found")
        _lib.hipGetErrorString.restype = ctypes.c_char_p
    return _lib


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: {lib().hipGetErrorString(rc).decode()}")


def set_device(d):
    check(lib().hipSetDevice(ctypes.c_int(d)), "hipSetDevice")


def malloc(nbytes):
    p = ctypes.c_void_p()
    check(lib().hipMalloc(ctypes.byref(p), ctypes.c_size_t(max(1, nbytes))), "hipMalloc")
    return p.value


def free(p):
    check(lib().hipFree(ctypes.c_void_p(p)), "hipFree")


def h2d(dst, arr):
    """numpy array -> device pointer (synchronous)."""
    import numpy as np
    a = np.ascontiguousarray(arr)
    check(lib().hipMemcpy(ctypes.c_void_p(dst), a.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(a.nbytes), 1),
          "hipMemcpy H2D")


def d2h(src, like):
    """device pointer -> a new numpy array shaped / typed like `like`."""
    import numpy as np
    out = np.empty_like(like)
    check(lib().hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(src), ctypes.c_size_t(out.nbytes), 2),
          "hipMemcpy D2H")
    return out


def synchronize():
    check(lib().hipDeviceSynchronize(), "hipDeviceSynchronize")


def mem_info():
    """(free, total) bytes of the current device."""
    f, t = ctypes.c_size_t(), ctypes.c_size_t()
    check(lib().hipMemGetInfo(ctypes.byref(f), ctypes.byref(t)), "hipMemGetInfo")
    return f.value, t.value


def memset(p, value, nbytes):
    check(lib().hipMemset(ctypes.c_void_p(p), ctypes.c_int(value), ctypes.c_size_t(nbytes)), "hipMemset")
    synchronize()


def stream_create():
    """A new (blocking) stream: the caller's stream of a test."""
    s = ctypes.c_void_p()
    check(lib().hipStreamCreate(ctypes.byref(s)), "hipStreamCreate")
    return s.value


def stream_synchronize(s):
    check(lib().hipStreamSynchronize(ctypes.c_void_p(s)), "hipStreamSynchronize")


def stream_destroy(s):
    check(lib().hipStreamDestroy(ctypes.c_void_p(s)), "hipStreamDestroy")
