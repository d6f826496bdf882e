// capi.cc — C-ABI over Context / PlanExecutor; no exception crosses it.
#include <chrono>
#include <cstring>
#include <list>
#include <memory>
#include <string>
#include <vector>

#include "gloo_amd.h"
#include "gloo_amd/common.h"
#include "gloo_amd/context.h"
#include "gloo_amd/errors.h"
#include "gloo_amd/executor.h"
#include "gloo_amd/ipc.h"
#include "gloo_amd/signal.h"
#include "gloo_amd/transport.h"

struct gloo_hip_context {
  std::shared_ptr<gloo_amd::Context> ctx;
  // function-style allreduce: one executor per option set, least recently
  // used first (every rank makes the same calls, so hits and evictions agree)
  std::list<std::pair<std::string, std::unique_ptr<gloo_amd::PlanExecutor>>> cache;
  gloo_amd::PlanExecutor* last = nullptr;  // the executor of the latest function-style call
};
struct gloo_hip_algorithm {
  std::unique_ptr<gloo_amd::PlanExecutor> exec;
};
struct gloo_hip_transport {
  std::unique_ptr<gloo_amd::transport::Device> dev;
};
struct gloo_hip_buffer {
  std::unique_ptr<gloo_amd::transport::Buffer> buf;
};
struct gloo_hip_ubuf {
  std::unique_ptr<gloo_amd::transport::UnboundBuffer> buf;
};

namespace {
template <typename F>
int guarded(F&& f) {
  try {
    f();
    return GLOO_HIP_OK;
  } catch (const gloo_amd::IoException& e) {
    return gloo_amd::setError(GLOO_HIP_EIO, std::string("IoException: ") + e.what());
  } catch (const std::exception& e) {
    return gloo_amd::setError(GLOO_HIP_EINVAL_ARG, e.what());
  } catch (...) {
    return gloo_amd::setError(GLOO_HIP_EINVAL_ARG, "unknown exception");
  }
}

// Function-style collectives: one executor per option set (the plan depends
// on sizes, not pointers; every rank makes the same calls, so hits and
// evictions agree), rebound to the call's buffers and run.
void runCached(gloo_hip_context_t ctx, int algo, int op, int dtype, const std::vector<void*>& ins,
               const std::vector<void*>& outs, size_t elements, size_t maxSeg, uint32_t tag,
               gloo_hip_stream_t stream, const std::vector<int>& extra) {
  // The key holds what the schedule depends on, never a rank-local value
  // such as the stream: ranks that pass different streams for the same call
  // must still hit and evict alike (their construction and tear-down are
  // collective).  The stream is rebound per call, like the buffers.
  std::string key = gloo_amd::strcat_(algo, "/", op, "/", dtype, "/", ins.size(), "/", outs.size(), "/", elements,
                                      "/", maxSeg, "/", tag);
  for (int v : extra) key += gloo_amd::strcat_("/", v);
  auto& cache = ctx->cache;
  auto it = cache.begin();
  for (; it != cache.end(); ++it)
    if (it->first == key) break;
  if (it == cache.end()) {
    constexpr size_t kMaxCached = 16;
    if (cache.size() == kMaxCached) cache.pop_back();
    cache.emplace_front(key, gloo_amd::PlanExecutor::create(ctx->ctx, algo, op, dtype, outs, elements,
                                                                      extra, static_cast<hipStream_t>(stream), ins,
                                                                      maxSeg));
    it = cache.begin();
  } else if (it != cache.begin()) {
    cache.splice(cache.begin(), cache, it);
    it = cache.begin();
  }
  it->second->setStream(static_cast<hipStream_t>(stream));
  it->second->setBuffers(ins, outs);
  ctx->last = it->second.get();
  it->second->run();
}
}  // namespace

extern "C" {

int gloo_hip_context_create(int rank, int size, const char* store_url, int device, int timeout_ms,
                            gloo_hip_context_t* out) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(out && store_url, "null argument");
    auto c = std::make_unique<gloo_hip_context>();
    c->ctx = std::make_shared<gloo_amd::Context>(
        rank, size, std::chrono::milliseconds(timeout_ms > 0 ? timeout_ms : 30000));
    c->ctx->connect(gloo_amd::openStore(store_url), device);
    *out = c.release();
  });
}

int gloo_hip_context_create_ex(int rank, int size, int device, int timeout_ms, gloo_hip_allgather_fn allgather,
                               void* user, gloo_hip_context_t* out) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(out && allgather, "null argument");
    auto c = std::make_unique<gloo_hip_context>();
    c->ctx = std::make_shared<gloo_amd::Context>(
        rank, size, std::chrono::milliseconds(timeout_ms > 0 ? timeout_ms : 30000));
    c->ctx->connect(std::make_shared<gloo_amd::CallbackStore>(allgather, user), device);
    *out = c.release();
  });
}

int gloo_hip_context_destroy(gloo_hip_context_t ctx) {
  return guarded([&] {
    if (ctx) ctx->cache.clear();  // executors tear down before the context
    delete ctx;
  });
}

int gloo_hip_algorithm_create_ws(gloo_hip_context_t ctx, int algo, int op, int dtype, void* const* ptrs, int nptrs,
                                 size_t count, const int* recv_elems, gloo_hip_stream_t stream, int workspace,
                                 gloo_hip_algorithm_t* out) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(ctx && out && ptrs && nptrs >= 1, "bad arguments");
    std::vector<int> re;
    if (algo == GLOO_HIP_ALGO_REDUCE_SCATTER) {
      GLOO_AMD_ENFORCE(recv_elems, "reduce-scatter needs recv_elems");
      re.assign(recv_elems, recv_elems + ctx->ctx->size);
    }
    if (algo == GLOO_HIP_ALGO_BCUBE && recv_elems) re.assign(recv_elems, recv_elems + 1);  // {base}
    auto a = std::make_unique<gloo_hip_algorithm>();
    a->exec = gloo_amd::PlanExecutor::create(ctx->ctx, algo, op, dtype,
                                                       std::vector<void*>(ptrs, ptrs + nptrs), count, re,
                                                       static_cast<hipStream_t>(stream), std::vector<void*>{}, 0,
                                                       workspace);
    *out = a.release();
  });
}

int gloo_hip_algorithm_create_streams(gloo_hip_context_t ctx, int algo, int op, int dtype, void* const* ptrs,
                                      int nptrs, size_t count, const int* recv_elems,
                                      const gloo_hip_stream_t* streams, int nstreams, int workspace,
                                      gloo_hip_algorithm_t* out) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(ctx && out && ptrs && nptrs >= 1, "bad arguments");
    // gloo/cuda_allreduce_ring_chunked.cc:55-58
    GLOO_AMD_ENFORCE(nstreams == 0 || (streams && nstreams == nptrs), "streams: ", nstreams, ", pointers: ", nptrs,
                     " (one stream per pointer, or none)");
    std::vector<int> re;
    if (algo == GLOO_HIP_ALGO_REDUCE_SCATTER) {
      GLOO_AMD_ENFORCE(recv_elems, "reduce-scatter needs recv_elems");
      re.assign(recv_elems, recv_elems + ctx->ctx->size);
    }
    if (algo == GLOO_HIP_ALGO_BCUBE && recv_elems) re.assign(recv_elems, recv_elems + 1);  // {base}
    std::vector<hipStream_t> ss;
    for (int i = 0; i < nstreams; i++) ss.push_back(static_cast<hipStream_t>(streams[i]));
    // Validated before the collective construction: a refusal after it would
    // run the executor's release() on this rank alone, and the peers would
    // wait at its barrier until the context timeout.
    for (hipStream_t t : ss)
      GLOO_AMD_ENFORCE(t != nullptr || ss.size() == 1, "null stream in a list of ", ss.size(),
                       " (one stream per pointer)");
    auto a = std::make_unique<gloo_hip_algorithm>();
    a->exec = gloo_amd::PlanExecutor::create(ctx->ctx, algo, op, dtype, std::vector<void*>(ptrs, ptrs + nptrs), count,
                                             re, ss.empty() ? nullptr : ss[0], std::vector<void*>{}, 0, workspace);
    if (ss.size() > 1) a->exec->setStreams(ss);
    *out = a.release();
  });
}

int gloo_hip_algorithm_set_streams(gloo_hip_algorithm_t a, const gloo_hip_stream_t* streams, int nstreams) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(a && (nstreams == 0 || streams), "bad arguments");
    std::vector<hipStream_t> ss;
    for (int i = 0; i < nstreams; i++) ss.push_back(static_cast<hipStream_t>(streams[i]));
    a->exec->setStreams(ss);
  });
}

int gloo_hip_algorithm_create(gloo_hip_context_t ctx, int algo, int op, int dtype, void* const* ptrs, int nptrs,
                              size_t count, const int* recv_elems, gloo_hip_stream_t stream,
                              gloo_hip_algorithm_t* out) {
  return gloo_hip_algorithm_create_ws(ctx, algo, op, dtype, ptrs, nptrs, count, recv_elems, stream,
                                      GLOO_HIP_WORKSPACE_DEVICE, out);
}

int gloo_hip_interp_batches(const gloo_hip_interp_desc_t* steps, int n, int* defer_out) {
  if (n < 0 || (n > 0 && (!steps || !defer_out)))
    return gloo_amd::setError(GLOO_HIP_EINVAL_ARG, "gloo_hip_interp_batches: bad arguments");
  return guarded([&] {
    std::vector<gloo_amd::InterpStep> v((size_t)n);
    for (int i = 0; i < n; i++) {
      const gloo_hip_interp_desc_t& d = steps[i];
      GLOO_AMD_ENFORCE(d.kind >= gloo_amd::kInterpCopy && d.kind <= gloo_amd::kInterpFold && d.nsrc >= 0 &&
                           d.nsrc <= GLOO_HIP_MAX_SRCS,
                       "gloo_hip_interp_batches: bad step ", i);
      gloo_amd::InterpStep& t = v[(size_t)i];
      std::memset(&t, 0, sizeof t);
      t.kind = d.kind;
      t.nsrc = d.kind == gloo_amd::kInterpFold ? d.nsrc : 1;
      t.dst = reinterpret_cast<char*>(d.dst);
      for (int j = 0; j < GLOO_HIP_MAX_SRCS; j++) t.src[j] = reinterpret_cast<const char*>(d.src[j]);
      t.n = d.bytes;
    }
    gloo_amd::markInterpBatches(v.data(), v.size(), 1);
    for (int i = 0; i < n; i++) defer_out[i] = v[(size_t)i].flags & gloo_amd::kInterpDefer ? 1 : 0;
  });
}

int gloo_hip_ipc_stats(uint64_t* out) {
  return gloo_hip_ipc_stats_ex(out, 5);
}

int gloo_hip_ipc_stats_ex(uint64_t* out, size_t n) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(out, "null argument");
    const gloo_amd::ipc::Stats st = gloo_amd::ipc::stats();
    const uint64_t v[] = {st.slabs, st.slabBytes, st.free, st.imports, st.opens, st.dropped};
    for (size_t i = 0; i < n && i < sizeof(v) / sizeof(v[0]); i++) out[i] = v[i];
  });
}

int gloo_hip_algorithm_run(gloo_hip_algorithm_t a) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(a, "null algorithm");
    a->exec->run();
  });
}

int gloo_hip_algorithm_destroy(gloo_hip_algorithm_t a) {
  return guarded([&] { delete a; });
}

int gloo_hip_allreduce(gloo_hip_context_t ctx, const gloo_hip_allreduce_options_t* o) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(ctx && o, "null argument");
    GLOO_AMD_ENFORCE(o->algorithm == 0 || o->algorithm == GLOO_HIP_ALLREDUCE_RING ||
                         o->algorithm == GLOO_HIP_ALLREDUCE_BCUBE,
                     "Algorithm not handled.");  // gloo/allreduce.cc:142-143
    GLOO_AMD_ENFORCE(o->noutputs >= 1 && o->outputs, "need at least one output");
    GLOO_AMD_ENFORCE(o->ninputs == 0 || o->inputs, "null inputs");
    if (o->elements == 0) return;  // gloo/allreduce.cc:98-100
    std::vector<void*> ins(o->inputs, o->inputs + o->ninputs), outs(o->outputs, o->outputs + o->noutputs);
    const int algo = o->algorithm == GLOO_HIP_ALLREDUCE_BCUBE ? GLOO_HIP_ALGO_ALLREDUCE_BCUBE
                                                              : GLOO_HIP_ALGO_ALLREDUCE_RING;
    runCached(ctx, algo, o->op, o->dtype, ins, outs, o->elements, o->max_segment_bytes, o->tag, o->stream, {});
  });
}

int gloo_hip_reduce_to_root(gloo_hip_context_t ctx, const gloo_hip_reduce_options_t* o) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(ctx && o, "null argument");
    if (o->elements == 0) return;  // gloo/reduce.cc:22-24
    GLOO_AMD_ENFORCE(o->output, "null output");
    GLOO_AMD_ENFORCE(o->root >= 0 && o->root < ctx->ctx->size, "root ", o->root, " out of range");  // :32
    std::vector<void*> ins, outs{o->output};
    if (o->input && o->input != o->output) ins.push_back(o->input);  // :46-48
    runCached(ctx, GLOO_HIP_ALGO_REDUCE, o->op, o->dtype, ins, outs, o->elements, o->max_segment_bytes, o->tag,
              o->stream, {o->root});
  });
}

double gloo_hip_algorithm_wait_seconds(gloo_hip_algorithm_t a) { return a ? a->exec->lastWaitSeconds() : 0.0; }

int gloo_hip_algorithm_set_profiling(gloo_hip_algorithm_t a, int on) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(a, "null algorithm");
    // 1: HIP events around every chunk reduction (eager runs);
    // 2: device stamps inside the kernels (graph replay kept)
    a->exec->setProfiling(on == 1);
    a->exec->setStamping(on == 2);
  });
}

int gloo_hip_algorithm_stats(gloo_hip_algorithm_t a, double* stats) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(a && stats, "null argument");
    stats[0] = a->exec->lastReduceSeconds();
    stats[1] = a->exec->lastReduceBytes();
    stats[2] = (double)a->exec->lastReduceCount();
    stats[3] = a->exec->lastWaitSeconds();
  });
}

namespace {
void modeOf(const gloo_amd::PlanExecutor& e, int* mode) {
  mode[0] = e.deviceSignalling() ? 1 : 0;
  mode[1] = e.hostArena() ? 2 : e.fineGrainedArena() ? 1 : 0;
  mode[2] = (e.foldSendUsed() ? 2 : 0) | (e.ownStream() ? 4 : 0);
  mode[3] = e.graphed() ? 1 : e.interpreted() ? 1 + e.interpSlices() : 0;
  gloo_amd::setError(0, e.graphError().empty() ? "" : "graph capture abandoned: " + e.graphError());
}
}  // namespace

int gloo_hip_algorithm_mode(gloo_hip_algorithm_t a, int* mode) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(a && mode, "null argument");
    modeOf(*a->exec, mode);
  });
}

int gloo_hip_context_mode(gloo_hip_context_t ctx, int* mode) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(ctx && mode, "null argument");
    GLOO_AMD_ENFORCE(ctx->last, "no function-style call on this context yet");
    modeOf(*ctx->last, mode);
  });
}

int gloo_hip_context_create_kv(int rank, int size, int device, int timeout_ms, gloo_hip_kv_set_fn set,
                               gloo_hip_kv_get_fn get, void* user, gloo_hip_context_t* out) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(out && set && get, "null argument");
    auto c = std::make_unique<gloo_hip_context>();
    c->ctx = std::make_shared<gloo_amd::Context>(
        rank, size, std::chrono::milliseconds(timeout_ms > 0 ? timeout_ms : 30000));
    c->ctx->connect(std::make_shared<gloo_amd::KvCallbackStore>(set, get, user), device);
    *out = c.release();
  });
}

int gloo_hip_transport_create(gloo_hip_context_t ctx, gloo_hip_stream_t stream, gloo_hip_transport_t* out) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(ctx && out, "null argument");
    auto t = std::make_unique<gloo_hip_transport>();
    t->dev = std::make_unique<gloo_amd::transport::Device>(ctx->ctx, static_cast<hipStream_t>(stream));
    *out = t.release();
  });
}

int gloo_hip_transport_destroy(gloo_hip_transport_t t) {
  return guarded([&] { delete t; });
}

int gloo_hip_buffer_create(gloo_hip_transport_t t, int peer, int slot, void* ptr, size_t size, int is_send,
                           gloo_hip_buffer_t* out) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(t && out, "null argument");
    auto& pair = t->dev->getPair(peer);
    auto b = std::make_unique<gloo_hip_buffer>();
    b->buf = is_send ? pair.createSendBuffer(slot, ptr, size) : pair.createRecvBuffer(slot, ptr, size);
    *out = b.release();
  });
}

int gloo_hip_buffer_destroy(gloo_hip_buffer_t b) {
  return guarded([&] { delete b; });
}

int gloo_hip_buffer_send(gloo_hip_buffer_t b, size_t offset, size_t length, size_t roffset) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(b, "null buffer");
    b->buf->send(offset, length, roffset);
  });
}

int gloo_hip_buffer_wait_recv(gloo_hip_buffer_t b) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(b, "null buffer");
    b->buf->waitRecv();
  });
}

int gloo_hip_buffer_wait_send(gloo_hip_buffer_t b) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(b, "null buffer");
    b->buf->waitSend();
  });
}

int gloo_hip_ubuf_create(gloo_hip_transport_t t, void* ptr, size_t size, gloo_hip_ubuf_t* out) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(t && out && (ptr || size == 0), "bad arguments");
    auto b = std::make_unique<gloo_hip_ubuf>();
    b->buf = std::make_unique<gloo_amd::transport::UnboundBuffer>(t->dev.get(), ptr, size);
    *out = b.release();
  });
}

int gloo_hip_ubuf_destroy(gloo_hip_ubuf_t b) {
  return guarded([&] { delete b; });
}

int gloo_hip_ubuf_send(gloo_hip_ubuf_t b, int dst, uint64_t slot, size_t offset, size_t nbytes) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(b, "null buffer");
    b->buf->send(dst, slot, offset, nbytes);
  });
}

int gloo_hip_ubuf_recv(gloo_hip_ubuf_t b, const int* srcs, int nsrcs, uint64_t slot, size_t offset, size_t nbytes) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(b && srcs && nsrcs > 0, "bad arguments");
    b->buf->recv(std::vector<int>(srcs, srcs + nsrcs), slot, offset, nbytes);
  });
}

namespace {
int waitResult(int rc, bool done) { return rc == GLOO_HIP_OK && !done ? 1 : rc; }
}  // namespace

int gloo_hip_ubuf_wait_recv(gloo_hip_ubuf_t b, int* rank, int timeout_ms) {
  bool done = false;
  const int rc = guarded([&] {
    GLOO_AMD_ENFORCE(b, "null buffer");
    done = b->buf->waitRecv(rank, std::chrono::milliseconds(timeout_ms));
  });
  return waitResult(rc, done);
}

int gloo_hip_ubuf_wait_send(gloo_hip_ubuf_t b, int* rank, int timeout_ms) {
  bool done = false;
  const int rc = guarded([&] {
    GLOO_AMD_ENFORCE(b, "null buffer");
    done = b->buf->waitSend(rank, std::chrono::milliseconds(timeout_ms));
  });
  return waitResult(rc, done);
}

int gloo_hip_ubuf_abort_wait_recv(gloo_hip_ubuf_t b) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(b, "null buffer");
    b->buf->abortWaitRecv();
  });
}

int gloo_hip_ubuf_abort_wait_send(gloo_hip_ubuf_t b) {
  return guarded([&] {
    GLOO_AMD_ENFORCE(b, "null buffer");
    b->buf->abortWaitSend();
  });
}

}  // extern "C"
