// newstyle_test.cc — TEST PROGRAM (built by oracle/Makefile where the
// reference sources exist; the binary travels to the GPU box, the reference
// does not).
//
// A Gloo program that fills the reference's own gloo::AllreduceOptions /
// gloo::ReduceOptions with DEVICE pointers, exactly as it would for
// gloo::allreduce / gloo::reduce (gloo/allreduce.h:89-193, gloo/reduce.h:19-110),
// and hands them to gloo::hip::allreduce / gloo::hip::reduce
// (gloo_amd/include/gloo_amd/gloo_collectives.h).  Ranks are threads, each
// with a gloo::rendezvous::Context over the reference's TCP transport
// (gloo/test/base_test.h:107-152).  The reduce function is the reference's
// gloo::sum / product / max / min<T> (gloo/math.h:15-73), so op and element
// type come from it as they would for a real caller.
//
// Usage: newstyle_test DIR [MODE]
//   MODE device (default): gloo::hip::allreduce / reduce on device buffers
//        over a TCP gloo::Context;
//   MODE hip-transport-host: the reference's OWN gloo::allreduce /
//        gloo::reduce (gloo/allreduce.cc, gloo/reduce.cc, unmodified) on host
//        buffers, over a gloo::Context whose pairs are the hip transport
//        (gloo_transport.h: its unbound buffers carry the messages).
//   DIR/meta.txt  "kind op dtype P nin nout n root seg"
//                 kind: ring | bcube | reduce; root: reduce only; seg: the
//                 maximum segment size in bytes (0: the default)
//   DIR/init.bin  P x nout x n elements: each rank's initial outputs
//   DIR/in.bin    P x nin x n elements: each rank's separate inputs (nin > 0)
// Every rank calls the collective TWICE (the second call reuses the cached
// schedule with fresh buffers) and writes DIR/out_<rank>_<call>.bin
// (nout x n elements; reduce: n).  tests/test_gloo_collectives.py compares
// them with the reference's goldens.
#include <hip/hip_runtime_api.h>

#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "gloo/rendezvous/context.h"
#include "gloo/rendezvous/hash_store.h"
#include "gloo/transport/tcp/device.h"
#include "gloo_amd/gloo_collectives.h"
#include "gloo_amd/gloo_transport.h"

namespace {

#define HIPOK(x)                                                                                    \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct Meta {
  std::string kind, op, dtype;
  int P = 0, nin = 0, nout = 0, root = 0;
  size_t n = 0, seg = 0;
};

std::vector<char> readFile(const std::string& f) {
  std::ifstream i(f, std::ios::binary);
  if (!i) return {};
  return std::vector<char>((std::istreambuf_iterator<char>(i)), std::istreambuf_iterator<char>());
}

void writeFile(const std::string& f, const void* p, size_t n) {
  std::ofstream o(f, std::ios::binary);
  o.write(static_cast<const char*>(p), (std::streamsize)n);
}

template <typename T>
gloo::hip::detail::ReduceFn opFn(const std::string& op) {
  using F = gloo::hip::detail::ReduceFn;
  if (op == "sum") return static_cast<F>(&gloo::sum<T>);
  if (op == "product") return static_cast<F>(&gloo::product<T>);
  if (op == "max") return static_cast<F>(&gloo::max<T>);
  if (op == "min") return static_cast<F>(&gloo::min<T>);
  throw std::runtime_error("unknown op " + op);
}

template <typename T>
std::string run(const Meta& m, const std::string& dir, bool hipHost) {
  const size_t bytes = m.n * sizeof(T);
  const std::vector<char> init = readFile(dir + "/init.bin");
  const std::vector<char> in = m.nin ? readFile(dir + "/in.bin") : std::vector<char>();
  if (init.size() != (size_t)m.P * m.nout * bytes || in.size() != (size_t)m.P * m.nin * bytes)
    return "init.bin / in.bin sizes do not match meta.txt";
  auto store = std::make_shared<gloo::rendezvous::HashStore>();
  std::mutex em;
  std::string err;
  std::vector<std::thread> ts;
  for (int rank = 0; rank < m.P; rank++) {
    ts.emplace_back([&, rank] {
      try {
        HIPOK(hipSetDevice(0));
        auto ctx = std::make_shared<gloo::rendezvous::Context>(rank, m.P);
        ctx->setTimeout(std::chrono::milliseconds(60000));
        std::shared_ptr<gloo::transport::Device> dev;
        if (hipHost) {
          gloo::transport::hip::attr a;
          a.device = 0;
          dev = gloo::transport::hip::CreateDevice(a);
        } else {
          gloo::transport::tcp::attr attr("localhost");
          dev = gloo::transport::tcp::CreateDevice(attr);
        }
        ctx->connectFullMesh(store, dev);
        for (int call = 0; call < 2; call++) {
          std::vector<T*> outs(m.nout), ins(m.nin);
          std::vector<std::vector<char>> hostBufs;  // hip-transport-host: the buffers themselves
          auto make = [&](const char* src) -> T* {
            if (hipHost) {
              hostBufs.emplace_back(src, src + bytes);
              hostBufs.back().resize(std::max<size_t>(bytes, 1));
              return reinterpret_cast<T*>(hostBufs.back().data());
            }
            T* p = nullptr;
            HIPOK(hipMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(bytes, 1)));
            HIPOK(hipMemcpy(p, src, bytes, hipMemcpyHostToDevice));
            return p;
          };
          hostBufs.reserve(m.nout + m.nin);
          for (int j = 0; j < m.nout; j++) outs[j] = make(init.data() + ((size_t)rank * m.nout + j) * bytes);
          for (int j = 0; j < m.nin; j++) ins[j] = make(in.data() + ((size_t)rank * m.nin + j) * bytes);
          std::vector<char> host((size_t)m.nout * bytes);
          if (m.kind == "reduce") {
            gloo::ReduceOptions opts(ctx);
            if (m.nin) opts.setInput(ins[0], m.n);
            opts.setOutput(outs[0], m.n);
            opts.setRoot(m.root);
            opts.setReduceFunction(opFn<T>(m.op));
            if (m.seg) opts.setMaxSegmentSize(m.seg);
            opts.setTag(7);
            if (hipHost) gloo::reduce(opts);
            else gloo::hip::reduce(opts);
          } else {
            gloo::AllreduceOptions opts(ctx);
            opts.setAlgorithm(m.kind == "bcube" ? gloo::AllreduceOptions::Algorithm::BCUBE
                                                : gloo::AllreduceOptions::Algorithm::RING);
            if (m.nin) opts.setInputs(ins, m.n);
            opts.setOutputs(outs, m.n);
            opts.setReduceFunction(opFn<T>(m.op));
            if (m.seg) opts.setMaxSegmentSize(m.seg);
            opts.setTag(7);
            if (hipHost) gloo::allreduce(opts);
            else gloo::hip::allreduce(opts);
          }
          for (int j = 0; j < m.nout; j++) {
            if (hipHost) std::memcpy(host.data() + (size_t)j * bytes, outs[j], bytes);
            else HIPOK(hipMemcpy(host.data() + (size_t)j * bytes, outs[j], bytes, hipMemcpyDeviceToHost));
          }
          writeFile(dir + "/out_" + std::to_string(rank) + "_" + std::to_string(call) + ".bin", host.data(),
                    host.size());
          if (!hipHost) {
            for (T* p : outs) HIPOK(hipFree(p));
            for (T* p : ins) HIPOK(hipFree(p));
          }
        }
        gloo::hip::releaseContext(ctx);  // collective, while the gloo::Context lives
        // every rank is done with the pairs before any tears its context down
        std::vector<char> one{1};
        store->set("done/" + std::to_string(rank), one);
        for (int r = 0; r < m.P; r++) store->wait({"done/" + std::to_string(r)});
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> lk(em);
        if (err.empty()) err = "rank " + std::to_string(rank) + ": " + e.what();
      }
    });
  }
  for (auto& t : ts) t.join();
  return err;
}

}  // namespace

// One case directory (meta.txt, init.bin, in.bin) -> its out_*.bin files;
// returns the error ("" on success).
std::string runDir(const std::string& dir, bool hh, Meta* mo) {
  Meta m;
  {
    std::istringstream s(std::string(readFile(dir + "/meta.txt").data(), readFile(dir + "/meta.txt").size()));
    s >> m.kind >> m.op >> m.dtype >> m.P >> m.nin >> m.nout >> m.n >> m.root >> m.seg;
    if (!s) return "bad meta.txt";
  }
  *mo = m;
  std::string err;
  try {
    if (m.dtype == "f32") err = run<float>(m, dir, hh);
    else if (m.dtype == "f64") err = run<double>(m, dir, hh);
    else if (m.dtype == "f16") err = run<gloo::float16>(m, dir, hh);
    else if (m.dtype == "bf16") err = run<c10::BFloat16>(m, dir, hh);
    else if (m.dtype == "i8") err = run<int8_t>(m, dir, hh);
    else if (m.dtype == "u8") err = run<uint8_t>(m, dir, hh);
    else if (m.dtype == "i32") err = run<int32_t>(m, dir, hh);
    else if (m.dtype == "i64") err = run<int64_t>(m, dir, hh);
    else if (m.dtype == "u64") err = run<uint64_t>(m, dir, hh);
    else err = "unknown dtype " + m.dtype;
  } catch (const std::exception& e) {
    err = e.what();
  }
  return err;
}

// newstyle_test DIR [MODE]            one case
// newstyle_test --batch LIST [MODE]   every case directory named in LIST (one
//                                     per line) in this one process; each gets
//                                     a result.txt ("ok" or "FAIL <why>")
int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: newstyle_test DIR [MODE] | --batch LIST [MODE]\n");
    return 2;
  }
  const bool batch = std::string(argv[1]) == "--batch";
  if (batch && argc < 3) return 2;
  const std::string mode = argc > (batch ? 3 : 2) ? argv[batch ? 3 : 2] : "device";
  if (mode != "device" && mode != "hip-transport-host") {
    std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 2;
  }
  const bool hh = mode == "hip-transport-host";
  std::vector<std::string> dirs;
  if (batch) {
    std::istringstream list(std::string(readFile(argv[2]).data(), readFile(argv[2]).size()));
    for (std::string line; std::getline(list, line);)
      if (!line.empty()) dirs.push_back(line);
  } else {
    dirs.push_back(argv[1]);
  }
  int failed = 0;
  for (const std::string& dir : dirs) {
    Meta m;
    const std::string err = runDir(dir, hh, &m);
    std::printf("%s %s/%s/%s/P%d\n%s\n", err.empty() ? "ok  " : "FAIL", m.kind.c_str(), m.op.c_str(), m.dtype.c_str(),
                m.P, err.c_str());
    std::fflush(stdout);
    if (batch) {
      std::FILE* f = std::fopen((dir + "/result.txt").c_str(), "w");
      if (f) {
        std::fprintf(f, "%s%s%s\n", err.empty() ? "ok" : "FAIL ", err.c_str(), "");
        std::fclose(f);
      }
    }
    failed += !err.empty();
  }
  return failed ? 1 : 0;
}
