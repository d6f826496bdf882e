"""gloo_amd — MI355X-native per-chunk reduction for Gloo (Python binding).

The product is the HIP library gloo_amd/libgloo_amd.so (C-ABI declared in
include/gloo_amd.h, kernels in gloo_amd/csrc/reduce.hip) and the C++ host
headers under gloo_amd/include/gloo_amd/.  This module is a thin ctypes
binding of that C-ABI for tests, smoke and the benchmark.  There is no CPU
fallback: if the library is missing, importing this package raises.

Mirrors the reference's reduction-function surface:
  ReductionType            gloo/algorithm.h:49-57
  ReductionFunction.call   gloo/algorithm.h:75-77  (dst = dst op src)
  CudaReductionFunction    gloo/cuda.h:286-358      (device overload, async)
"""
import ctypes
import enum
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# GLOO_AMD_LIB: another build of the same library (A/B measurements of
# compile-time kernel variants, tools/build_fold_variants.sh)
LIB_PATH = os.environ.get("GLOO_AMD_LIB") or os.path.join(_HERE, "libgloo_amd.so")


class ReductionType(enum.IntEnum):
    """gloo::ReductionType (gloo/algorithm.h:49-57)."""
    SUM = 1
    PRODUCT = 2
    MAX = 3
    MIN = 4


class DType(enum.IntEnum):
    I8 = 0
    U8 = 1
    I32 = 2
    U32 = 3
    I64 = 4
    U64 = 5
    F16 = 6
    BF16 = 7
    F32 = 8
    F64 = 9


DTYPE_NAMES = {"i8": DType.I8, "u8": DType.U8, "i32": DType.I32, "u32": DType.U32,
               "i64": DType.I64, "u64": DType.U64, "f16": DType.F16, "bf16": DType.BF16,
               "f32": DType.F32, "f64": DType.F64}
OP_NAMES = {"sum": ReductionType.SUM, "product": ReductionType.PRODUCT,
            "max": ReductionType.MAX, "min": ReductionType.MIN}

EXPORTED = ("gloo_hip_reduce", "gloo_hip_reduce3", "gloo_hip_reduce_multi",
            "gloo_hip_dtype_size", "gloo_hip_last_error", "gloo_hip_version",
            "gloo_hip_set_variant", "gloo_hip_plan", "gloo_hip_reduce_staged", "gloo_hip_register_op",
            "gloo_hip_copy_kernel", "gloo_hip_copy_kernel_multi")


class GlooHipError(RuntimeError):
    """Raised when a gloo_hip_* call returns a non-zero status
    (the Python face of GLOO_ENFORCE / EnforceNotMet, gloo/common/logging.h:32-59)."""

    def __init__(self, code, msg):
        super().__init__(f"gloo_hip error {code}: {msg}")
        self.code = code


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (there is deliberately no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    L.gloo_hip_reduce.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, sz, vp]
    L.gloo_hip_reduce3.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, vp, sz, vp]
    L.gloo_hip_reduce_multi.argtypes = [ctypes.c_int, ctypes.c_int, vp,
                                        ctypes.POINTER(vp), ctypes.c_int, sz, vp]
    L.gloo_hip_dtype_size.argtypes = [ctypes.c_int]
    L.gloo_hip_dtype_size.restype = sz
    L.gloo_hip_last_error.restype = ctypes.c_char_p
    L.gloo_hip_version.restype = ctypes.c_char_p
    L.gloo_hip_set_variant.argtypes = [ctypes.c_int]
    L.gloo_hip_reduce_staged.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, sz, vp, vp, sz, vp]
    L.gloo_hip_register_op.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_int)]
    L.gloo_hip_copy_kernel.argtypes = [vp, vp, sz, ctypes.c_uint, vp]
    L.gloo_hip_copy_kernel_multi.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(sz), ctypes.c_int,
                                             ctypes.c_uint, vp]
    return L


lib = _load()


def _check(rc):
    if rc != 0:
        raise GlooHipError(rc, lib.gloo_hip_last_error().decode(errors="replace"))


def _as_op(op):
    return int(OP_NAMES[op]) if isinstance(op, str) else int(op)  # ints: built-in or registered (>= 1000)


def _as_dtype(dtype):
    return int(DTYPE_NAMES[dtype]) if isinstance(dtype, str) else int(dtype)


def dtype_size(dtype):
    return lib.gloo_hip_dtype_size(_as_dtype(dtype))


def version():
    return lib.gloo_hip_version().decode()


# ---- raw-pointer API (device pointers as ints, stream as int handle) -------

def reduce_ptr(op, dtype, dst, src, n, stream=0):
    """dst[i] = dst[i] op src[i] on device pointers (async on `stream`)."""
    _check(lib.gloo_hip_reduce(_as_op(op), _as_dtype(dtype), dst, src, n, stream or None))


def reduce3_ptr(op, dtype, c, a, b, n, stream=0):
    """c[i] = a[i] op b[i] on device pointers (async on `stream`)."""
    _check(lib.gloo_hip_reduce3(_as_op(op), _as_dtype(dtype), c, a, b, n, stream or None))


def reduce_multi_ptr(op, dtype, dst, srcs, n, stream=0):
    arr = (ctypes.c_void_p * len(srcs))(*srcs)
    _check(lib.gloo_hip_reduce_multi(_as_op(op), _as_dtype(dtype), dst, arr, len(srcs), n,
                                     stream or None))


def reduce_staged(op, dtype, host_dst, host_src, n, dev_dst, dev_src, piece_elems=0, stream=0):
    """Host-staged chunk reduction (gloo_hip_reduce_staged): host_dst op=
    host_src, zero-copy over PCIe when both host buffers are pinned and
    mapped and piece_elems is 0, else staged through the device scratch,
    pipelined in pieces of at least 16 MiB (one pass for a smaller chunk)."""
    _check(lib.gloo_hip_reduce_staged(_as_op(op), _as_dtype(dtype), host_dst, host_src, n, dev_dst, dev_src,
                                      piece_elems, stream or None))


def register_op(fn_ptr, user=None):
    """gloo_hip_register_op: a caller-supplied device reduction (a C function
    pointer, as int, of type gloo_hip_custom_fn) -> an op code >= 1000
    (gloo::ReductionType::CUSTOM, gloo/algorithm.h:49-57) accepted by every
    entry point that takes `op`."""
    out = ctypes.c_int()
    _check(lib.gloo_hip_register_op(ctypes.c_void_p(fn_ptr), user, ctypes.byref(out)))
    return out.value


def copy_kernel(dst, src, nbytes, blocks=0, stream=0):
    """gloo_hip_copy_kernel: the SEND steps' kernel copy engine."""
    _check(lib.gloo_hip_copy_kernel(dst, src, nbytes, blocks, stream or None))


def copy_kernel_multi(dsts, srcs, nbytes, blocks=0, stream=0):
    """gloo_hip_copy_kernel_multi: several copies in one launch (a mesh
    schedule's sends to every peer); nbytes is one size or one per copy."""
    n = len(dsts)
    sizes = list(nbytes) if hasattr(nbytes, "__len__") else [nbytes] * n
    vp = ctypes.c_void_p
    _check(lib.gloo_hip_copy_kernel_multi((vp * n)(*dsts), (vp * n)(*srcs), (ctypes.c_size_t * n)(*sizes), n,
                                          blocks, stream or None))


def set_variant(v):
    """Measurement knob: fp32 SUM kernel variant (0 = tuned default)."""
    return lib.gloo_hip_set_variant(int(v))


# ---- torch-tensor convenience (device memory / streams come from torch) -----

def _torch_dtype_code(t):
    import torch
    m = {torch.int8: DType.I8, torch.uint8: DType.U8, torch.int32: DType.I32,
         torch.int64: DType.I64, torch.float16: DType.F16, torch.bfloat16: DType.BF16,
         torch.float32: DType.F32, torch.float64: DType.F64}
    if hasattr(torch, "uint32"):
        m[torch.uint32] = DType.U32
    if hasattr(torch, "uint64"):
        m[torch.uint64] = DType.U64
    if t.dtype not in m:
        raise TypeError(f"unsupported dtype {t.dtype}")
    return m[t.dtype]


def _stream_handle(t, stream):
    import torch
    if stream is None:
        stream = torch.cuda.current_stream(t.device)
    return stream.cuda_stream


def reduce(op, dst, src, stream=None):
    """In-place dst op= src for contiguous same-dtype device tensors —
    CudaReductionFunction<T>::call(dst, src, n, stream) (gloo/cuda.h:326-333)."""
    if dst.dtype != src.dtype or dst.numel() != src.numel():
        raise ValueError("dst/src must have equal dtype and numel")
    if not (dst.is_cuda and src.is_cuda and dst.is_contiguous() and src.is_contiguous()):
        raise ValueError("dst/src must be contiguous device tensors")
    reduce_ptr(op, _torch_dtype_code(dst), dst.data_ptr(), src.data_ptr(), dst.numel(),
               _stream_handle(dst, stream))
    return dst


def reduce3(op, c, a, b, stream=None):
    """c = a op b for contiguous device tensors (gloo::sum<T>(c, a, b, n) shape)."""
    if not (c.dtype == a.dtype == b.dtype) or not (c.numel() == a.numel() == b.numel()):
        raise ValueError("c/a/b must have equal dtype and numel")
    reduce3_ptr(op, _torch_dtype_code(c), c.data_ptr(), a.data_ptr(), b.data_ptr(), c.numel(),
                _stream_handle(c, stream))
    return c


class ReductionFunction:
    """Python face of HipReductionFunction<T> (C++: gloo_amd/include/gloo_amd/hip.h),
    itself the MI355X twin of CudaReductionFunction<T> (gloo/cuda.h:286-358)."""

    def __init__(self, rtype):
        self.rtype = ReductionType(rtype)

    def type(self):
        return self.rtype

    def call(self, dst, src, n=None, stream=None):
        if n is None:
            return reduce(self.rtype, dst, src, stream)
        return reduce(self.rtype, dst[:n], src[:n], stream)


ReductionFunction.sum = ReductionFunction(ReductionType.SUM)
ReductionFunction.product = ReductionFunction(ReductionType.PRODUCT)
ReductionFunction.max = ReductionFunction(ReductionType.MAX)
ReductionFunction.min = ReductionFunction(ReductionType.MIN)


# ---- contexts and algorithms (GPU allreduce / reduce-scatter drop-ins) -----

ALGORITHMS = {"ring_chunked": 0, "halving_doubling": 1, "ring": 2, "local": 3,
              "reduce_scatter": 4, "bcube": 10}  # bcube: AllreduceBcube, recv_elems = [base]


def _bind_collectives(L):
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    L.gloo_hip_context_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                          ctypes.c_int, ctypes.POINTER(vp)]
    L.gloo_hip_context_destroy.argtypes = [vp]
    L.gloo_hip_algorithm_create.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.POINTER(vp), ctypes.c_int, sz,
                                            ctypes.POINTER(ctypes.c_int), vp, ctypes.POINTER(vp)]
    L.gloo_hip_algorithm_create_ws.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.POINTER(vp), ctypes.c_int, sz,
                                               ctypes.POINTER(ctypes.c_int), vp, ctypes.c_int, ctypes.POINTER(vp)]
    L.gloo_hip_algorithm_create_streams.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                    ctypes.POINTER(vp), ctypes.c_int, sz,
                                                    ctypes.POINTER(ctypes.c_int), ctypes.POINTER(vp), ctypes.c_int,
                                                    ctypes.c_int, ctypes.POINTER(vp)]
    L.gloo_hip_algorithm_set_streams.argtypes = [vp, ctypes.POINTER(vp), ctypes.c_int]
    L.gloo_hip_ipc_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    L.gloo_hip_ipc_stats_ex.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t]
    L.gloo_hip_algorithm_run.argtypes = [vp]
    L.gloo_hip_algorithm_destroy.argtypes = [vp]
    L.gloo_hip_algorithm_wait_seconds.argtypes = [vp]
    L.gloo_hip_algorithm_wait_seconds.restype = ctypes.c_double
    L.gloo_hip_algorithm_set_profiling.argtypes = [vp, ctypes.c_int]
    L.gloo_hip_algorithm_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
    L.gloo_hip_algorithm_mode.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
    L.gloo_hip_context_mode.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]


_bind_collectives(lib)
EXPORTED = EXPORTED + ("gloo_hip_context_create", "gloo_hip_context_create_ex", "gloo_hip_context_destroy",
                       "gloo_hip_algorithm_create", "gloo_hip_algorithm_run",
                       "gloo_hip_algorithm_destroy", "gloo_hip_algorithm_wait_seconds",
                       "gloo_hip_algorithm_set_profiling", "gloo_hip_algorithm_stats",
                       "gloo_hip_algorithm_mode", "gloo_hip_algorithm_create_ws", "gloo_hip_context_mode",
                       "gloo_hip_algorithm_create_streams", "gloo_hip_algorithm_set_streams", "gloo_hip_ipc_stats",
                       "gloo_hip_ipc_stats_ex")
# the xGMI transport's bound buffers (gloo_amd/include/gloo_amd/gloo_transport.h)
EXPORTED = EXPORTED + ("gloo_hip_context_create_kv", "gloo_hip_transport_create", "gloo_hip_transport_destroy",
                       "gloo_hip_buffer_create", "gloo_hip_buffer_destroy", "gloo_hip_buffer_send",
                       "gloo_hip_buffer_wait_recv", "gloo_hip_buffer_wait_send",
                       # unbound buffers (gloo/transport/unbound_buffer.h) on the same transport
                       "gloo_hip_ubuf_create", "gloo_hip_ubuf_destroy", "gloo_hip_ubuf_send", "gloo_hip_ubuf_recv",
                       "gloo_hip_ubuf_wait_recv", "gloo_hip_ubuf_wait_send", "gloo_hip_ubuf_abort_wait_recv",
                       "gloo_hip_ubuf_abort_wait_send")

WORKSPACES = {"device": 0, "host": 1}


def _bind_transport(L):
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    L.gloo_hip_transport_create.argtypes = [vp, vp, ctypes.POINTER(vp)]
    L.gloo_hip_transport_destroy.argtypes = [vp]
    L.gloo_hip_buffer_create.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, sz, ctypes.c_int, ctypes.POINTER(vp)]
    L.gloo_hip_buffer_destroy.argtypes = [vp]
    L.gloo_hip_buffer_send.argtypes = [vp, sz, sz, sz]
    L.gloo_hip_buffer_wait_recv.argtypes = [vp]
    L.gloo_hip_buffer_wait_send.argtypes = [vp]


_bind_transport(lib)


class Transport:
    """The xGMI transport's bound buffers (gloo::transport::Pair /
    Buffer, gloo/transport/pair.h:33-41, buffer.h:26-34) over a Context:
    construction is collective.  Receive buffers in device memory are written
    in place by the peer (across processes: the allocation shared as a dma-buf
    and mapped by the sender, any size); host receive buffers across processes,
    of any length, through a landing segment in node shared memory, copied
    into the buffer at wait_recv."""

    def __init__(self, ctx, stream=0):
        h = ctypes.c_void_p()
        _check(lib.gloo_hip_transport_create(ctx._h, stream or None, ctypes.byref(h)))
        self._h = h

    def buffer(self, peer, slot, ptr, size, send):
        return TransportBuffer(self, peer, slot, ptr, size, send)

    def close(self):
        if self._h:
            _check(lib.gloo_hip_transport_destroy(self._h))
            self._h = None


class TransportBuffer:
    def __init__(self, t, peer, slot, ptr, size, send):
        h = ctypes.c_void_p()
        _check(lib.gloo_hip_buffer_create(t._h, peer, slot, ptr or None, size, 1 if send else 0, ctypes.byref(h)))
        self._h = h

    def send(self, offset=0, length=None, roffset=0):
        _check(lib.gloo_hip_buffer_send(self._h, offset, length if length is not None else 0, roffset))

    def wait_recv(self):
        _check(lib.gloo_hip_buffer_wait_recv(self._h))

    def wait_send(self):
        _check(lib.gloo_hip_buffer_wait_send(self._h))

    def close(self):
        if self._h:
            _check(lib.gloo_hip_buffer_destroy(self._h))
            self._h = None


def ipc_stats():
    """This process's pool of cross-process slabs (gloo_amd/include/gloo_amd/ipc.h:
    HIP VMM blocks, never freed while the process lives, reused by size
    class): slabs exported and their bytes, slabs free for reuse, peer slabs
    mapped, imports made, mappings of exited peers dropped."""
    out = (ctypes.c_uint64 * 6)()
    _check(lib.gloo_hip_ipc_stats_ex(out, 6))
    return {"slabs": out[0], "slab_bytes": out[1], "free": out[2], "peer_slabs_mapped": out[3],
            "imports": out[4], "dropped": out[5]}


def _mode_dict(out):
    err = lib.gloo_hip_last_error()
    err = err.decode() if isinstance(err, bytes) else (err or "")
    return {"device_signal": bool(out[0]), "fine_arena": out[1] == 1,
            "host_arena": out[1] == 2, "fold_send": bool(out[2] & 2), "own_stream": bool(out[2] & 4),
            "graph": out[3] == 1, "interp": out[3] >= 2, "interp_slices": max(0, out[3] - 1),
            "graph_error": err[len("graph capture abandoned: "):]
            if err.startswith("graph capture abandoned: ") else ""}


class Context:
    """rendezvous::Context(rank, size) + connectFullMesh(store, device)
    (gloo/rendezvous/context.cc:25-35).  store_url: "file:<dir>" when ranks
    are processes, "mem:<name>" when ranks are threads of one process."""

    def __init__(self, rank, size, store_url, device=0, timeout_ms=30000):
        self.rank, self.size = rank, size
        h = ctypes.c_void_p()
        _check(lib.gloo_hip_context_create(rank, size, store_url.encode(), device, timeout_ms,
                                           ctypes.byref(h)))
        self._h = h

    def last_mode(self):
        """How the latest function-style call (allreduce / reduce_to_root)
        on this context ran (see Algorithm.mode)."""
        out = (ctypes.c_int * 4)()
        _check(lib.gloo_hip_context_mode(self._h, out))
        return _mode_dict(out)

    def close(self):
        if self._h:
            _check(lib.gloo_hip_context_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Algorithm:
    """A constructed GPU algorithm (CudaAllreduceRingChunked & co.); run() is
    Algorithm::run() (gloo/algorithm.h:26).  ptrs: device pointers (ints).
    workspace: "device" (inboxes in HBM) or "host" (pinned host-memory
    inboxes, the CudaHostWorkspace placement; gloo/cuda_workspace.h:20-31)."""

    def __init__(self, ctx, algo, op, dtype, ptrs, count, recv_elems=None, stream=0, workspace="device",
                 streams=None, base=None):
        """stream: one stream for the plan (0: the algorithm's own stream,
        and run() returns with outputs complete).  streams: one stream handle per
        pointer instead (the reference's `streams` argument,
        gloo/cuda_allreduce_ring_chunked.cc:55-67): run() orders pointer i
        after the work queued on streams[i], and every streams[i] after the
        collective.  base: AllreduceBcube's group size (gloo::Context::base,
        gloo/context.h:28-33), the same as recv_elems=[base]."""
        self.ctx = ctx
        if base is not None:
            recv_elems = [int(base)]
        arr = (ctypes.c_void_p * len(ptrs))(*ptrs)
        rp = None
        if recv_elems is not None:
            rp = (ctypes.c_int * len(recv_elems))(*[int(x) for x in recv_elems])
        h = ctypes.c_void_p()
        a = ALGORITHMS[algo] if isinstance(algo, str) else int(algo)
        ws = WORKSPACES[workspace] if isinstance(workspace, str) else int(workspace)
        if streams is not None:
            sarr = (ctypes.c_void_p * max(1, len(streams)))(*[int(x) for x in streams])
            _check(lib.gloo_hip_algorithm_create_streams(ctx._h, a, _as_op(op), _as_dtype(dtype), arr, len(ptrs),
                                                         int(count), rp, sarr, len(streams), ws, ctypes.byref(h)))
        else:
            _check(lib.gloo_hip_algorithm_create_ws(ctx._h, a, _as_op(op), _as_dtype(dtype), arr, len(ptrs),
                                                    int(count), rp, stream or None, ws, ctypes.byref(h)))
        self._h = h

    def set_streams(self, streams):
        sarr = (ctypes.c_void_p * max(1, len(streams)))(*[int(x) for x in streams])
        _check(lib.gloo_hip_algorithm_set_streams(self._h, sarr, len(streams)))

    def run(self):
        _check(lib.gloo_hip_algorithm_run(self._h))

    def wait_seconds(self):
        return lib.gloo_hip_algorithm_wait_seconds(self._h)

    def set_profiling(self, on=True):
        """0/False: off; 1/True: HIP events around every chunk reduction
        (eager runs); 2: device stamps inside the reduce kernels (graph
        replay kept)."""
        mode = 2 if on == 2 and on is not True else 1 if on else 0
        _check(lib.gloo_hip_algorithm_set_profiling(self._h, mode))

    def stats(self):
        """After run(): reduce-kernel seconds, algorithmic bytes reduced, chunk
        reductions, host seconds blocked on peers (profiling must be on)."""
        out = (ctypes.c_double * 4)()
        _check(lib.gloo_hip_algorithm_stats(self._h, out))
        return {"reduce_s": out[0], "reduce_bytes": out[1], "reductions": int(out[2]), "wait_s": out[3]}

    def mode(self):
        """How run() executes: device-side signalling, fine-grained inboxes,
        kernel copy engine, hipGraph replay, one-launch plan interpreter;
        'graph_error' says why capture was abandoned (empty if it was not)."""
        out = (ctypes.c_int * 4)()
        _check(lib.gloo_hip_algorithm_mode(self._h, out))
        return _mode_dict(out)

    def close(self):
        if self._h:
            _check(lib.gloo_hip_algorithm_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- new-style function API: gloo::allreduce(opts) -------------------------

class AllreduceOptions(ctypes.Structure):
    """gloo_hip_allreduce_options_t (mirrors gloo::AllreduceOptions,
    gloo/allreduce.h:89-193)."""
    _fields_ = [("algorithm", ctypes.c_int), ("op", ctypes.c_int), ("dtype", ctypes.c_int),
                ("inputs", ctypes.POINTER(ctypes.c_void_p)), ("ninputs", ctypes.c_int),
                ("outputs", ctypes.POINTER(ctypes.c_void_p)), ("noutputs", ctypes.c_int),
                ("elements", ctypes.c_size_t), ("max_segment_bytes", ctypes.c_size_t),
                ("tag", ctypes.c_uint32), ("stream", ctypes.c_void_p)]


lib.gloo_hip_allreduce.argtypes = [ctypes.c_void_p, ctypes.POINTER(AllreduceOptions)]
EXPORTED = EXPORTED + ("gloo_hip_allreduce", "gloo_hip_plan_ex", "gloo_hip_interp_batches")


ALLREDUCE_ALGORITHMS = {"ring": 1, "bcube": 2}  # AllreduceOptions::Algorithm (gloo/allreduce.h:38-42)


def allreduce(ctx, outputs, elements, dtype, op="sum", inputs=None, max_segment_bytes=0, tag=0,
              stream=0, algorithm="ring"):
    """gloo::allreduce(opts) on device pointers, RING (gloo/allreduce.cc:147-392)
    or BCUBE (:397-669); every output receives the reduction of all inputs (or
    of the outputs when no inputs are given) over all ranks."""
    inputs = list(inputs or [])
    o = AllreduceOptions()
    o.algorithm = ALLREDUCE_ALGORITHMS[algorithm] if isinstance(algorithm, str) else int(algorithm)
    o.op = _as_op(op)
    o.dtype = _as_dtype(dtype)
    ins = (ctypes.c_void_p * max(1, len(inputs)))(*inputs)
    outs = (ctypes.c_void_p * len(outputs))(*outputs)
    o.inputs = ins if inputs else None
    o.ninputs = len(inputs)
    o.outputs = outs
    o.noutputs = len(outputs)
    o.elements = int(elements)
    o.max_segment_bytes = int(max_segment_bytes)
    o.tag = tag
    o.stream = stream or None
    _check(lib.gloo_hip_allreduce(ctx._h, ctypes.byref(o)))


# ---- new-style function API: gloo::reduce(opts) ----------------------------

class ReduceOptions(ctypes.Structure):
    """gloo_hip_reduce_options_t (mirrors gloo::ReduceOptions, gloo/reduce.h:19-110)."""
    _fields_ = [("op", ctypes.c_int), ("dtype", ctypes.c_int), ("input", ctypes.c_void_p),
                ("output", ctypes.c_void_p), ("elements", ctypes.c_size_t), ("root", ctypes.c_int),
                ("max_segment_bytes", ctypes.c_size_t), ("tag", ctypes.c_uint32), ("stream", ctypes.c_void_p)]


lib.gloo_hip_reduce_to_root.argtypes = [ctypes.c_void_p, ctypes.POINTER(ReduceOptions)]
EXPORTED = EXPORTED + ("gloo_hip_reduce_to_root",)


def reduce_to_root(ctx, output, elements, dtype, root, op="sum", input=None, max_segment_bytes=0, tag=0,
                   stream=0):
    """gloo::reduce(opts) (gloo/reduce.cc:21-247) on device pointers: the
    root's output receives the reduction of every rank's input (or output,
    when no input is given)."""
    o = ReduceOptions()
    o.op = _as_op(op)
    o.dtype = _as_dtype(dtype)
    o.input = input or None
    o.output = output
    o.elements = int(elements)
    o.root = int(root)
    o.max_segment_bytes = int(max_segment_bytes)
    o.tag = tag
    o.stream = stream or None
    _check(lib.gloo_hip_reduce_to_root(ctx._h, ctypes.byref(o)))
