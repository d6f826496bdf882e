/*
 * gloo_amd.h — C-ABI of the MI355X-native Gloo per-chunk reduction.
 *
 * This is the drop-in boundary for Gloo's hot path: the element-wise
 * sum / product / max / min that every allreduce / reduce-scatter schedule
 * applies to each arriving chunk.  Plain pointers, sizes and integer enums
 * only; no HIP, torch or C++ types cross this boundary, and no C++ exception
 * ever escapes it (every entry point returns a status code).
 *
 * Reference interfaces replaced (paths relative to facebookincubator/gloo):
 *   gloo_hip_reduce   <- gloo::cudaSum/cudaProduct/cudaMax/cudaMin<T>
 *                        (gloo/cuda.h:274-284, kernels gloo/cuda.cu:283-401),
 *                        i.e. the device overload of
 *                        CudaReductionFunction<T>::call (gloo/cuda.h:326-333):
 *                        dst[i] = dst[i] (op) src[i], async on `stream`.
 *   gloo_hip_reduce3  <- the 3-operand host form gloo::sum/product/max/min<T>
 *                        (void* c, const void* a, const void* b, size_t n)
 *                        (gloo/math.h:15-73), which is also the new-style
 *                        reduce `Func` signature (gloo/allreduce.h:36).
 *   gloo_hip_op_t     <- gloo::ReductionType (gloo/algorithm.h:49-57).
 *   gloo_hip_dtype_t  <- the union of the instantiation lists of
 *                        gloo/cuda.cu:265-272,394-401 and
 *                        gloo/test/math_test.cc:23-32.
 *
 * Semantics (bit-exact with gloo/math.h evaluated in the listed order):
 *   SUM      c = a + b      (integers wrap modulo 2^bits)
 *   PRODUCT  c = a * b      (integers wrap modulo 2^bits)
 *   MAX      c = (a < b) ? b : a      == std::max(a, b)  (gloo/math.h:51)
 *   MIN      c = (b < a) ? b : a      == std::min(a, b)  (gloo/math.h:66)
 *   For the in-place form a := dst, b := src, so a NaN already in dst is kept
 *   and a NaN arriving in src is ignored by MAX/MIN, exactly as
 *   `if (src op dst) dst = src` in gloo/cuda.cu:337-355.
 *   f16 / bf16: both operands widened to f32, op in f32, rounded back to
 *   nearest-even (gloo/math.cc:17-97 F16C path; c10::BFloat16 for bf16);
 *   MAX/MIN compare in f32 and copy the raw 16-bit operand.
 *
 * Buffers may start at any element-aligned address and `c` may alias `a`
 * (the in-place call).  n may be 0.  The functions never allocate, free or
 * synchronise: they enqueue one kernel on `stream` and return.
 */
#ifndef GLOO_AMD_H_
#define GLOO_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Mirrors gloo::ReductionType (gloo/algorithm.h:49-57). */
typedef enum {
  GLOO_HIP_SUM = 1,
  GLOO_HIP_PRODUCT = 2,
  GLOO_HIP_MAX = 3,
  GLOO_HIP_MIN = 4,
} gloo_hip_op_t;

typedef enum {
  GLOO_HIP_I8 = 0,
  GLOO_HIP_U8 = 1,
  GLOO_HIP_I32 = 2,
  GLOO_HIP_U32 = 3,
  GLOO_HIP_I64 = 4,
  GLOO_HIP_U64 = 5,
  GLOO_HIP_F16 = 6,
  GLOO_HIP_BF16 = 7,
  GLOO_HIP_F32 = 8,
  GLOO_HIP_F64 = 9,
  GLOO_HIP_NUM_DTYPES = 10,
} gloo_hip_dtype_t;

/* Status codes: 0 = success, > 0 = a hipError_t, < 0 = argument error. */
#define GLOO_HIP_OK 0
#define GLOO_HIP_EINVAL_OP (-1)
#define GLOO_HIP_EINVAL_DTYPE (-2)
#define GLOO_HIP_EINVAL_PTR (-3)
#define GLOO_HIP_EINVAL_ARG (-4)
#define GLOO_HIP_EIO (-5) /* a peer did not answer within the context timeout (gloo::IoException) */

/* A hipStream_t passed as an opaque pointer (NULL = the default stream). */
typedef void* gloo_hip_stream_t;

/* In-place per-chunk reduction: dst[i] = dst[i] (op) src[i], i < n.
 * Replaces cudaSum/cudaProduct/cudaMax/cudaMin<T> (gloo/cuda.cu:283-401). */
int gloo_hip_reduce(int op, int dtype, void* dst, const void* src, size_t n,
                    gloo_hip_stream_t stream);

/* Three-operand form: c[i] = a[i] (op) b[i]; c may alias a or b.
 * Replaces gloo::sum/product/max/min<T>(c, a, b, n) (gloo/math.h:15-73). */
int gloo_hip_reduce3(int op, int dtype, void* c, const void* a, const void* b,
                     size_t n, gloo_hip_stream_t stream);

/* Multi-source local reduction: dst[i] = (((srcs[0][i] op srcs[1][i]) op
 * srcs[2][i]) ... op srcs[k-1][i]), left to right, in ONE pass over HBM.
 * dst may alias srcs[0].  This is the fused form of the reference's local
 * multi-pointer loop `for i in 1..k: fn(ptrs[0], ptrs[i], count)`
 * (gloo/allreduce_local.cc:28-33, gloo/allreduce_ring_chunked.h:89-91),
 * bit-identical to it because the association order is the same.
 * k must be in [1, GLOO_HIP_MAX_SRCS]; srcs is a HOST array of k device
 * pointers. */
#define GLOO_HIP_MAX_SRCS 8
int gloo_hip_reduce_multi(int op, int dtype, void* dst,
                          const void* const* srcs, int k, size_t n,
                          gloo_hip_stream_t stream);

/* Host-staged chunk reduction: host_dst[i] = host_dst[i] (op) host_src[i]
 * for a chunk that starts and ends in (pinned) host memory — a transport's
 * receive buffer — computed by the HIP kernel through device scratch
 * dev_dst / dev_src (n elements each, caller-owned).  piece_elems = 0:
 * when both host buffers are pinned AND mapped (hipHostGetDevicePointer
 * succeeds), one kernel reduces them in place over PCIe (zero-copy, the
 * scratch is unused, the fastest way measured); otherwise, and for any
 * piece_elems > 0, the chunk is staged through the scratch in pieces of
 * max(piece_elems, 16 MiB) elements' bytes: H2D of piece k+1, the kernel of
 * piece k and D2H of piece k-1 overlap on per-thread copy streams (smaller
 * pieces measured slower than one pass); a chunk of at most one piece goes
 * H2D, kernel, D2H in one pass on `stream`.  Ordered after the work already
 * on `stream`; the host result is complete once `stream` has drained.  The device side of the reference's CudaLocalHostReduce
 * (gloo/cuda_collectives_host.h:22-136), with the reduction on the GPU. */
int gloo_hip_reduce_staged(int op, int dtype, void* host_dst, const void* host_src, size_t n,
                           void* dev_dst, void* dev_src, size_t piece_elems, gloo_hip_stream_t stream);

/* Custom reductions: gloo::ReductionType::CUSTOM (= 1000) with a user
 * function (gloo/algorithm.h:49-95) and the new-style reduce `Func`
 * (gloo/allreduce.h:36), on device memory.  The function enqueues
 * c[i] = a[i] (op) b[i], i < n, on `stream` (c may alias a; it must not
 * allocate, free or synchronise — it may be captured into a hipGraph).
 * gloo_hip_register_op returns an op code >= GLOO_HIP_CUSTOM that every
 * entry point taking an `op` accepts.  Algorithms with a custom op run the
 * reference's own exchange routes (no mesh plans), call the function for
 * every REDUCE and FOLD step (a k-source fold as k - 1 calls, left to
 * right), and never use the fused or interpreted kernels. */
#define GLOO_HIP_CUSTOM 1000
typedef void (*gloo_hip_custom_fn)(void* user, void* c, const void* a, const void* b, size_t n,
                                   gloo_hip_stream_t stream);
int gloo_hip_register_op(gloo_hip_custom_fn fn, void* user, int* op_out);

/* The kernel copy engine of a plan's SEND steps (copy_signal_kernel
 * without a flag): dst[0, bytes) = src[0, bytes) in 16-byte packets at any
 * relative misalignment, with `blocks` workgroups (0: one per 16 KiB tile,
 * capped at 1024).  Exported for measurement tools (blit vs kernel copies;
 * DESIGN.md §4) and callers that want a copy with no DMA-engine dependence. */
int gloo_hip_copy_kernel(void* dst, const void* src, size_t bytes, unsigned blocks, gloo_hip_stream_t stream);

/* (new, measurement) Up to 8 such copies in ONE launch, all in flight together
 * — the mesh schedules' sends to every peer (one xGMI link each): copy j gets
 * at most `blocks` workgroups (0: 64, the executor's per-peer default). */
int gloo_hip_copy_kernel_multi(void* const* dsts, const void* const* srcs, const size_t* bytes, int n,
                               unsigned blocks, gloo_hip_stream_t stream);

/* Size in bytes of one element of `dtype`, or 0 when dtype is unknown. */
size_t gloo_hip_dtype_size(int dtype);

/* Human-readable text of the last error raised on the calling thread. */
const char* gloo_hip_last_error(void);

/* Library version, "MAJOR.MINOR.PATCH". */
const char* gloo_hip_version(void);

/* Tuning knob for the measurement harness: select the kernel variant used by
 * the fp32 SUM path.  0 = default (tuned).  Returns the previous value. */
int gloo_hip_set_variant(int variant);

/* ------------------------------------------------------------------------
 * Schedules.  Each of the reference's reducing algorithms is restated as a
 * per-rank PLAN: the exact sequence of one-sided sends, receive waits,
 * reductions, copies and notifications its run() performs (same offsets,
 * lengths, peers, order — hence the same association order and bit-identical
 * results).  The HIP executor (gloo_hip_algo_*) walks a plan over device
 * memory; tests simulate all ranks' plans on the CPU against golden vectors.
 * ---------------------------------------------------------------------- */
typedef enum {
  GLOO_HIP_ALGO_RING_CHUNKED = 0,     /* gloo/allreduce_ring_chunked.h        */
  GLOO_HIP_ALGO_HALVING_DOUBLING = 1, /* gloo/allreduce_halving_doubling.h    */
  GLOO_HIP_ALGO_RING = 2,             /* gloo/allreduce_ring.h                */
  GLOO_HIP_ALGO_LOCAL = 3,            /* gloo/allreduce_local.{h,cc}          */
  GLOO_HIP_ALGO_REDUCE_SCATTER = 4,   /* gloo/reduce_scatter.h (HD)           */
  GLOO_HIP_ALGO_ALLREDUCE_RING = 5,   /* new-style gloo::allreduce(opts), RING
                                         (gloo/allreduce.cc:147-392)          */
  /* AllreduceRingChunked's RESULT with mesh data movement: each chunk pair
   * goes straight from every rank to the rank where the ring finishes it,
   * over all xGMI links at once, and is folded there in the ring's exact
   * association and operand order (bit-identical), then sent to every rank.
   * 2 <= size <= GLOO_HIP_MAX_SRCS.  RING_CHUNKED executes as this plan in
   * that range unless GLOO_AMD_MESH=0. */
  GLOO_HIP_ALGO_RING_CHUNKED_MESH = 6,
  GLOO_HIP_ALGO_ALLREDUCE_BCUBE = 7,  /* new-style gloo::allreduce(opts), BCUBE
                                         (gloo/allreduce.cc:397-669)          */
  GLOO_HIP_ALGO_REDUCE = 8,           /* new-style gloo::reduce(opts)
                                         (gloo/reduce.cc:21-247); the root is
                                         recv_elems[0] in gloo_hip_plan*      */
  /* AllreduceRingChunked's own ring route (its hops, association and bytes)
   * with three inboxes per channel, so that each round's reduce and the send
   * of its result run as one pass (plan.cc planRingChunkedPipe).  RING_CHUNKED
   * executes as this plan wherever it keeps the ring route (GLOO_AMD_MESH=0
   * or size > GLOO_HIP_MAX_SRCS) with a built-in op; a custom op keeps the
   * literal ring order. */
  GLOO_HIP_ALGO_RING_CHUNKED_PIPE = 9,
  /* AllreduceBcube (gloo/allreduce_bcube.h) and its GPU twin
   * CudaAllreduceBcube (gloo/cuda_allreduce_bcube.{h,cc}): groups of `base`
   * ranks, log_base(P) reduce-scatter steps and the all-gather back.  The
   * base (gloo::Context::base, gloo/context.h:28-33; 0 or absent = 2) is
   * recv_elems[0] in gloo_hip_plan* and gloo_hip_algorithm_create.  For
   * 2 <= size <= 8 it executes as its derived mesh plan (| GLOO_HIP_ALGO_MESH)
   * wherever every rank ends with the same expression trees (P a power of
   * the base, counts of about P and more), else on the reference's route. */
  GLOO_HIP_ALGO_BCUBE = 10,
} gloo_hip_algo_t;

/* algo | GLOO_HIP_ALGO_MESH: the algorithm's result with mesh data movement,
 * derived mechanically (gloo_amd/csrc/mesh.cc): every rank's plan is run
 * symbolically to find, per element range, the exact expression tree the
 * reference evaluates and the rank that finishes it; raw pieces then go
 * straight to that rank (all links at once), which evaluates the same tree,
 * and (allreduce) sends the result to every rank.  Bit-identical results.
 * For HALVING_DOUBLING and REDUCE_SCATTER (and RING_CHUNKED), 2 <= size <= 8. */
#define GLOO_HIP_ALGO_MESH 0x100

typedef enum {
  GLOO_HIP_STEP_DECL_RECV = 0,   /* inbox region for (peer, slot): arena[dst_off, +length) */
  GLOO_HIP_STEP_SEND = 1,        /* src[src_off, +length) -> peer's (me, slot) region       */
  GLOO_HIP_STEP_WAIT_RECV = 2,   /* wait for the next message from (peer, slot)             */
  GLOO_HIP_STEP_REDUCE = 3,      /* user[dst_off..] = user[dst_off..] op arena[src_off..]   */
  GLOO_HIP_STEP_COPY = 4,        /* dst[dst_off..] = src[src_off..] (memmove semantics)     */
  GLOO_HIP_STEP_NOTIFY = 5,      /* one notification to (peer, slot)                        */
  GLOO_HIP_STEP_WAIT_NOTIFY = 6, /* wait for the next notification from (peer, slot)        */
  GLOO_HIP_STEP_WAIT_SEND = 7,   /* wait until our last send to (peer, slot) has completed  */
  GLOO_HIP_STEP_LOCAL_REDUCE = 8,/* ptrs[0] = ((ptrs[0] op ptrs[1]) op ...), length elts    */
  GLOO_HIP_STEP_LOCAL_BCAST = 9, /* ptrs[i] = ptrs[0] for i >= 1, length elements           */
  GLOO_HIP_STEP_FOLD_SRC = 10,   /* next source of the following FOLD: src[src_off..]        */
  GLOO_HIP_STEP_FOLD = 11,       /* user[dst_off, +length) = fold of the pending FOLD_SRCs:
                                    acc = s0; acc = acc op s_k (or s_k op acc with
                                    GLOO_HIP_FOLD_REVERSE), k = 1.. in order             */
} gloo_hip_step_kind_t;

/* Message channels between a pair of ranks (the reference's slot roles). */
#define GLOO_HIP_SLOT_DATA0 0
#define GLOO_HIP_SLOT_DATA1 1
#define GLOO_HIP_SLOT_NOTIFY 2
#define GLOO_HIP_SLOT_DIST 3
#define GLOO_HIP_SLOT_DIST_NOTIFY 4
#define GLOO_HIP_SLOT_AUX0 5
#define GLOO_HIP_SLOT_AUX1 6
#define GLOO_HIP_SLOT_AUX_NOTIFY 7
#define GLOO_HIP_NUM_SLOTS 8

/* flags: which space each side of a data step lives in. */
#define GLOO_HIP_SRC_ARENA 1 /* else the user buffer ptrs[0] */
#define GLOO_HIP_DST_ARENA 2
/* LOCAL_REDUCE over [dst_off, +length) folds the separate INPUT buffers into
 * output 0 (new-style allreduce; one input = copy), instead of folding the
 * outputs into output 0.  On REDUCE: user[dst] = input0[dst] op arena[src]
 * (gloo::reduce's out = in op tmp); on SEND: the source is input 0. */
#define GLOO_HIP_FROM_INPUTS 4
/* FOLD: each new source is the LEFT operand (acc = s_k op acc). */
#define GLOO_HIP_FOLD_REVERSE 8
/* FOLD: balanced pairwise tree over the sources in order (k a power of two):
 * ((s0 op s1) op (s2 op s3)) op ((s4 op s5) op (s6 op s7)).  FOLD also takes
 * GLOO_HIP_DST_ARENA (result into the arena). */
#define GLOO_HIP_FOLD_TREE 16
/* WAIT_NOTIFY: wait for the notification of the PREVIOUS run (a credit the
 * receiver returns after consuming; satisfied at once in the first run). */
#define GLOO_HIP_PREV_RUN 32

typedef struct {
  int32_t kind;
  int32_t peer;
  int32_t slot;
  int32_t flags;
  uint64_t dst_off; /* elements */
  uint64_t src_off; /* elements */
  uint64_t length;  /* elements */
} gloo_hip_step_t;

/* Build rank `rank`'s plan of algorithm `algo` for `size` ranks, `count`
 * elements and `nptrs` local pointers.  recv_elems (size entries) is used by
 * GLOO_HIP_ALGO_REDUCE_SCATTER only.  With steps == NULL only *nsteps is
 * filled.  *arena_elems receives the inbox arena size this rank needs. */
int gloo_hip_plan(int algo, int rank, int size, size_t count, int nptrs,
                  const int* recv_elems, gloo_hip_step_t* steps, size_t capacity,
                  size_t* nsteps, size_t* arena_elems);

/* Full form: `ninputs` separate input buffers (0 = the outputs are the
 * inputs), `noutputs` outputs, element size and the new-style allreduce's
 * maximum segment size in bytes (0 = 1 MiB, gloo/allreduce.h:78). */
int gloo_hip_plan_ex(int algo, int rank, int size, size_t count, int ninputs, int noutputs,
                     size_t elem_size, size_t max_segment_bytes, const int* recv_elems,
                     gloo_hip_step_t* steps, size_t capacity, size_t* nsteps,
                     size_t* arena_elems);

/* (new, tests and tooling) The batching rule of the one-launch plan
 * interpreter: which steps of a step list are not drained before the next
 * (signal.h kInterpDefer).  Each step is a kind (0 copy, 1 send, 2 signal,
 * 3 wait, 4 fold), its destination and nsrc source addresses and its length
 * in bytes; addresses are only compared, never dereferenced.  defer_out[i]
 * receives 1 where step i and step i+1 share one drain. */
typedef struct {
  int32_t kind;
  int32_t nsrc;
  uint64_t dst;
  uint64_t src[GLOO_HIP_MAX_SRCS];
  uint64_t bytes;
} gloo_hip_interp_desc_t;
int gloo_hip_interp_batches(const gloo_hip_interp_desc_t* steps, int n, int* defer_out);

/* ------------------------------------------------------------------------
 * Contexts and algorithms (the GPU allreduce / reduce-scatter drop-ins).
 *
 *   gloo_hip_context_create  <- rendezvous::Context(rank, size) +
 *                               connectFullMesh(store, device)
 *                               (gloo/rendezvous/context.cc:25-35); the store
 *                               is "file:<dir>" (ranks = processes of one
 *                               node) or "mem:<name>" (ranks = threads).
 *   gloo_hip_algorithm_create <- the constructors of CudaAllreduceRingChunked
 *                               (gloo/cuda_allreduce_ring_chunked.h:19-26),
 *                               CudaAllreduceHalvingDoubling
 *                               (gloo/cuda_allreduce_halving_doubling.h:25-30),
 *                               CudaAllreduceRing, CudaAllreduceLocal and
 *                               ReduceScatterHalvingDoubling
 *                               (gloo/reduce_scatter.h:112-117): device
 *                               pointers `ptrs` (nptrs of them, on this
 *                               rank's device), `count` elements each.
 *                               Collective: every rank creates its
 *                               algorithms in the same order.
 *   gloo_hip_algorithm_run   <- Algorithm::run() (gloo/algorithm.h:26).  With
 *                               stream == NULL outputs are complete on
 *                               return; otherwise the work is ordered on
 *                               `stream` and the caller synchronises.
 * ---------------------------------------------------------------------- */
typedef struct gloo_hip_context* gloo_hip_context_t;
typedef struct gloo_hip_algorithm* gloo_hip_algorithm_t;

int gloo_hip_context_create(int rank, int size, const char* store_url, int device,
                            int timeout_ms, gloo_hip_context_t* out);
int gloo_hip_context_destroy(gloo_hip_context_t ctx);

/* Bootstrap over an existing collective context instead of a store: the
 * caller supplies an all-gather of fixed `block`-byte records (every rank
 * passes `in`; `out` receives size * block bytes, rank r's record at
 * r * block; return 0 on success).  Every exchange the library makes (the
 * control block's name, each algorithm's inbox-arena / IPC records,
 * set-up and tear-down barriers) is one such collective call, made in the
 * same order on every rank from the calling thread.  This is how a Gloo
 * program hands over its own gloo::Context (gloo/context.h:26-59): the
 * header-only bridge gloo_amd/include/gloo_amd/gloo_bridge.h passes
 * gloo::allgather over that context's pairs, so there is no second
 * rendezvous. */
typedef int (*gloo_hip_allgather_fn)(void* user, const void* in, void* out, size_t block);
int gloo_hip_context_create_ex(int rank, int size, int device, int timeout_ms, gloo_hip_allgather_fn allgather,
                               void* user, gloo_hip_context_t* out);

int gloo_hip_algorithm_create(gloo_hip_context_t ctx, int algo, int op, int dtype,
                              void* const* ptrs, int nptrs, size_t count,
                              const int* recv_elems, gloo_hip_stream_t stream,
                              gloo_hip_algorithm_t* out);
/* Where the inboxes (the transport's receive buffers) live — the reference's
 * workspace template argument (gloo/cuda_workspace.h:20-31):
 *   DEVICE  HBM of the rank's GPU (CudaDeviceWorkspace; the default here);
 *   HOST    pinned host memory shared by the node's ranks (CudaHostWorkspace:
 *           chunks arrive in host memory, as from a socket/NIC); peers write
 *           them over PCIe and the reduce kernel reads them in place
 *           (zero-copy) while accumulating into the device buffer. */
typedef enum { GLOO_HIP_WORKSPACE_DEVICE = 0, GLOO_HIP_WORKSPACE_HOST = 1 } gloo_hip_workspace_t;

/* gloo_hip_algorithm_create with an explicit workspace. */
int gloo_hip_algorithm_create_ws(gloo_hip_context_t ctx, int algo, int op, int dtype, void* const* ptrs, int nptrs,
                                 size_t count, const int* recv_elems, gloo_hip_stream_t stream, int workspace,
                                 gloo_hip_algorithm_t* out);

/* gloo_hip_algorithm_create_ws with one stream per pointer, the reference's
 * `const std::vector<cudaStream_t>& streams` (gloo/cuda_allreduce_ring_chunked.h:19-26,
 * GLOO_ENFORCE_EQ(streams.size(), ptrs.size()) at .cc:55-58): nstreams is 0
 * (run() returns with the outputs complete) or nptrs.  run() orders its use
 * of ptrs[i] after the work already queued on streams[i], and on return
 * every streams[i] is ordered after the collective (docs/cuda.md:7-11): the
 * caller synchronises with any of them.  The library never uses a stream
 * outside create/run, so a caller may destroy it between runs (each run()
 * then needs the streams it was created with, or those of
 * gloo_hip_algorithm_set_streams). */
int gloo_hip_algorithm_create_streams(gloo_hip_context_t ctx, int algo, int op, int dtype, void* const* ptrs,
                                      int nptrs, size_t count, const int* recv_elems,
                                      const gloo_hip_stream_t* streams, int nstreams, int workspace,
                                      gloo_hip_algorithm_t* out);
/* Rebind the streams of later runs (same rule: 0 or nptrs of them). */
int gloo_hip_algorithm_set_streams(gloo_hip_algorithm_t algo, const gloo_hip_stream_t* streams, int nstreams);

int gloo_hip_algorithm_run(gloo_hip_algorithm_t algo);

/* This process's pool of cross-process slabs (gloo_amd/include/gloo_amd/ipc.h:
 * HIP VMM blocks shared as dma-buf fds, never freed while the process lives,
 * reused by size class; no reference counterpart, for tests and tools):
 * out5[0] = slabs exported, [1] = their bytes, [2] = slabs free for reuse,
 * [3] = peer slabs mapped, [4] = imports made (a peer slab is mapped once and
 * kept). */
int gloo_hip_ipc_stats(uint64_t* out5);
/* The same, up to 6 words: + mappings of exited peers (their pid reused)
 * dropped. */
int gloo_hip_ipc_stats_ex(uint64_t* out, size_t n);
int gloo_hip_algorithm_destroy(gloo_hip_algorithm_t algo);
/* Host seconds the last run() spent blocked waiting for peers. */
double gloo_hip_algorithm_wait_seconds(gloo_hip_algorithm_t algo);
/* Measurement.  on = 1: bracket every chunk reduction of run() with HIP
 * events (runs are then enqueued eagerly); on = 2: device-side stamps inside
 * the reduce kernels (each records its first-workgroup start and
 * last-workgroup end on the GPU's 100 MHz clock), which keeps hipGraph
 * replay; 0: off.  After a run: stats[0] = summed reduce-kernel seconds,
 * stats[1] = algorithmic bytes reduced (3 * n * sizeof(T) per two-operand
 * chunk, (k + 1) * n * sizeof(T) per k-source fold), stats[2] = chunk
 * reductions, stats[3] = host seconds blocked on peers. */
int gloo_hip_algorithm_set_profiling(gloo_hip_algorithm_t algo, int on);
int gloo_hip_algorithm_stats(gloo_hip_algorithm_t algo, double* stats4);

/* How the algorithm executes (no reference counterpart; for tests and
 * tools): mode4[0] = device-side signalling, [1] = inbox arena (0 device
 * memory no peer writes, 1 device fine-grained, 2 pinned host),
 * [2] = bit 1: some run fused a fold with the SENDs of its result
 * (fold+forward), bit 2: runs on the algorithm's own stream (run() returns
 * with the outputs complete), [3] = how run() launches the plan: 0 enqueued
 * step by step, 1 a captured hipGraph replayed, k >= 2 the one-launch plan
 * interpreter with k - 1 workgroups (> 1: sliced).  If graph capture was
 * abandoned, gloo_hip_last_error() says why. */
int gloo_hip_algorithm_mode(gloo_hip_algorithm_t algo, int* mode4);
/* The same for the schedule that ran the latest function-style call
 * (gloo_hip_allreduce / gloo_hip_reduce_to_root) on `ctx`. */
int gloo_hip_context_mode(gloo_hip_context_t ctx, int* mode4);

/* ------------------------------------------------------------------------
 * New-style function API: gloo::allreduce(const AllreduceOptions&)
 * (gloo/allreduce.h:89-193, gloo/allreduce.cc:97-145), RING algorithm.
 * inputs may be empty (the outputs are the inputs); every output receives
 * the result.  Collective: all ranks call with the same options in the same
 * order.  The first call with a given option set builds the schedule and
 * inbox arena (a store exchange); later calls reuse it with the buffers of
 * the call.
 * ---------------------------------------------------------------------- */
#define GLOO_HIP_ALLREDUCE_RING 1  /* AllreduceOptions::Algorithm::RING  */
#define GLOO_HIP_ALLREDUCE_BCUBE 2 /* AllreduceOptions::Algorithm::BCUBE (gloo/allreduce.h:38-42) */
typedef struct {
  int algorithm;            /* 0 (unspecified = RING), RING or BCUBE      */
  int op;                   /* gloo_hip_op_t: the reduce Func             */
  int dtype;                /* gloo_hip_dtype_t: setInputs<T>/setOutputs<T> */
  void* const* inputs;      /* device pointers, may be NULL               */
  int ninputs;
  void* const* outputs;     /* device pointers, at least one              */
  int noutputs;
  size_t elements;
  size_t max_segment_bytes; /* setMaxSegmentSize; 0 = 1 MiB               */
  uint32_t tag;             /* setTag                                     */
  gloo_hip_stream_t stream; /* NULL: outputs complete on return           */
} gloo_hip_allreduce_options_t;

int gloo_hip_allreduce(gloo_hip_context_t ctx, const gloo_hip_allreduce_options_t* opts);

/* ------------------------------------------------------------------------
 * New-style function API: gloo::reduce(ReduceOptions&) (gloo/reduce.h:19-112,
 * gloo/reduce.cc:21-247): a ring reduce-scatter over <= max_segment_bytes
 * segments, then every rank's reduced chunk is gathered at `root`.  `input`
 * may be NULL (the output is the input).  Only the root's output holds the
 * full result; the other ranks' outputs hold the same partial reductions the
 * reference leaves there.  Collective, cached per option set like
 * gloo_hip_allreduce.
 * ---------------------------------------------------------------------- */
typedef struct {
  int op;                   /* gloo_hip_op_t: the reduce Func              */
  int dtype;                /* gloo_hip_dtype_t: setInput<T>/setOutput<T>  */
  void* input;              /* device pointer, may be NULL                 */
  void* output;             /* device pointer                              */
  size_t elements;
  int root;                 /* setRoot                                     */
  size_t max_segment_bytes; /* setMaxSegmentSize; 0 = 1 MiB (reduce.h:98)  */
  uint32_t tag;             /* setTag                                      */
  gloo_hip_stream_t stream; /* NULL: the output is complete on return      */
} gloo_hip_reduce_options_t;

int gloo_hip_reduce_to_root(gloo_hip_context_t ctx, const gloo_hip_reduce_options_t* opts);

/* ------------------------------------------------------------------------
 * The xGMI transport: bound buffers of gloo::transport::Pair / Buffer
 * (gloo/transport/pair.h:33-41, gloo/transport/buffer.h:26-34) over device
 * memory.  gloo_amd/include/gloo_amd/gloo_transport.h wraps these into a
 * gloo::transport::Device (gloo/transport/device.h:34-54) that
 * gloo::rendezvous::Context::connectFullMesh accepts.
 *
 *   gloo_hip_context_create_kv  <- transport::Context::createAndConnectAllPairs
 *       (gloo/transport/context.cc:26-89): the caller's key/value store
 *       (gloo::IStore set / wait+get) carries the set-up records.  set: store
 *       `len` bytes under `key`; get: wait up to timeout_ms for `key`, copy up
 *       to `cap` bytes into `out` and its full length into *len (the library
 *       calls again with a larger buffer when *len > cap).  Both return 0 on
 *       success, nonzero on failure (a timeout: GLOO_HIP_EIO).  The store
 *       must outlive the context: receive buffers publish records in it.
 *   gloo_hip_transport_create   <- transport::Device::createContext: one per
 *       context (collective, in the same order as algorithm creation); sends
 *       are ordered on `stream` (NULL: a stream of its own).
 *   gloo_hip_buffer_create      <- Pair::createSendBuffer (is_send = 1) /
 *       createRecvBuffer (is_send = 0) for the pair to `peer`.  A receive
 *       buffer is memory the peer writes into: device memory (HIP IPC across
 *       processes, the pointer itself within one process) or host memory
 *       (written directly within one process; across processes carried in
 *       the channel's 48 payload bytes, the reference's notification
 *       buffers).  ptr == NULL / size 0: a notification buffer.  Any number
 *       of distinct slots may be live (up to 128 receive buffers per peer).
 *   gloo_hip_buffer_send        <- Buffer::send(offset, length, roffset): a
 *       copy into the peer's receive buffer (a direct xGMI copy between
 *       GPUs), then, stream-ordered after the bytes landed, an arrival.
 *   gloo_hip_buffer_wait_recv   <- Buffer::waitRecv: the next arrival, or
 *       GLOO_HIP_EIO after the context timeout (gloo::IoException).
 *   gloo_hip_buffer_wait_send   <- Buffer::waitSend: the last send's copy out
 *       of this buffer has completed.
 * ---------------------------------------------------------------------- */
typedef int (*gloo_hip_kv_set_fn)(void* user, const char* key, const void* data, size_t len);
typedef int (*gloo_hip_kv_get_fn)(void* user, const char* key, int timeout_ms, void* out, size_t cap, size_t* len);
int gloo_hip_context_create_kv(int rank, int size, int device, int timeout_ms, gloo_hip_kv_set_fn set,
                               gloo_hip_kv_get_fn get, void* user, gloo_hip_context_t* out);

typedef struct gloo_hip_transport* gloo_hip_transport_t;
typedef struct gloo_hip_buffer* gloo_hip_buffer_t;
int gloo_hip_transport_create(gloo_hip_context_t ctx, gloo_hip_stream_t stream, gloo_hip_transport_t* out);
int gloo_hip_transport_destroy(gloo_hip_transport_t t);
int gloo_hip_buffer_create(gloo_hip_transport_t t, int peer, int slot, void* ptr, size_t size, int is_send,
                           gloo_hip_buffer_t* out);
int gloo_hip_buffer_destroy(gloo_hip_buffer_t b);
int gloo_hip_buffer_send(gloo_hip_buffer_t b, size_t offset, size_t length, size_t roffset);
int gloo_hip_buffer_wait_recv(gloo_hip_buffer_t b);
int gloo_hip_buffer_wait_send(gloo_hip_buffer_t b);

/* Unbound buffers (gloo/transport/unbound_buffer.h:32-121) on the same
 * transport: two-sided send / recv matched per (source, slot) in order,
 * recv-from-any over `srcs`.  Sends are eager (the bytes are staged in node
 * shared memory at once, so waitSend never blocks); the receiver copies them
 * out in wait_recv.  Host or device memory.  nbytes = SIZE_MAX: the rest of
 * the buffer from offset.
 *   gloo_hip_ubuf_wait_recv / wait_send: 0 = done (*rank = the peer),
 *   1 = aborted (abort_wait_*), GLOO_HIP_EIO = timed out (timeout_ms < 0:
 *   the context's timeout). */
typedef struct gloo_hip_ubuf* gloo_hip_ubuf_t;
int gloo_hip_ubuf_create(gloo_hip_transport_t t, void* ptr, size_t size, gloo_hip_ubuf_t* out);
int gloo_hip_ubuf_destroy(gloo_hip_ubuf_t b);
int gloo_hip_ubuf_send(gloo_hip_ubuf_t b, int dst, uint64_t slot, size_t offset, size_t nbytes);
int gloo_hip_ubuf_recv(gloo_hip_ubuf_t b, const int* srcs, int nsrcs, uint64_t slot, size_t offset, size_t nbytes);
int gloo_hip_ubuf_wait_recv(gloo_hip_ubuf_t b, int* rank, int timeout_ms);
int gloo_hip_ubuf_wait_send(gloo_hip_ubuf_t b, int* rank, int timeout_ms);
int gloo_hip_ubuf_abort_wait_recv(gloo_hip_ubuf_t b);
int gloo_hip_ubuf_abort_wait_send(gloo_hip_ubuf_t b);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* GLOO_AMD_H_ */
