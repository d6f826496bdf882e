// store.h — rendezvous key/value stores (mirrors gloo::rendezvous::Store,
// gloo/rendezvous/store.h, FileStore gloo/rendezvous/file_store.h:19 and
// HashStore gloo/rendezvous/hash_store.h:20).  Used only at setup: to publish
// each rank's inbox arena (its pool slab: pid, incarnation, slab id) and the control block's name.
#pragma once

#include <chrono>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace gloo_amd {

class Store {
 public:
  virtual ~Store() = default;
  virtual void set(const std::string& key, const std::vector<char>& data) = 0;
  // Blocks until `key` exists (or throws IoException after `timeout`).
  virtual std::vector<char> get(const std::string& key, std::chrono::milliseconds timeout) = 0;
  // Collective: each of the `size` ranks contributes `mine` under a `tag`
  // unique to this call; returns every rank's blob in rank order.  Every
  // exchange gloo_amd makes is one of these (context connect, an
  // algorithm's arena records, barriers), so a store that can only all-gather
  // (CallbackStore) is enough.  Default: set(tag/rank) + get of every rank.
  virtual std::vector<std::vector<char>> allgather(const std::string& tag, int rank, int size,
                                                   const std::vector<char>& mine, std::chrono::milliseconds timeout);
};

// The all-gather of an existing collective context supplied by the caller:
// gloo_hip_context_create_ex, through which a Gloo program bootstraps over
// its own gloo::Context (gloo_amd/include/gloo_amd/gloo_bridge.h).  Fixed
// blocks of kBlock bytes per rank: a 4-byte length, then the blob.
class CallbackStore : public Store {
 public:
  using Fn = int (*)(void* user, const void* in, void* out, size_t block);
  static constexpr size_t kBlock = 4096;  // a segmented arena record is up to ~2 KiB (executor.cc)
  CallbackStore(Fn fn, void* user) : fn_(fn), user_(user) {}
  void set(const std::string& key, const std::vector<char>& data) override;
  std::vector<char> get(const std::string& key, std::chrono::milliseconds timeout) override;
  std::vector<std::vector<char>> allgather(const std::string& tag, int rank, int size, const std::vector<char>& mine,
                                           std::chrono::milliseconds timeout) override;

 private:
  Fn fn_;
  void* user_;
};

// The key/value store of a caller (gloo gloo::IStore behind
// gloo_hip_context_create_kv, gloo_amd/include/gloo_amd/gloo_transport.h):
// set, and a get that waits for the key up to a timeout.
class KvCallbackStore : public Store {
 public:
  using SetFn = int (*)(void* user, const char* key, const void* data, size_t len);
  using GetFn = int (*)(void* user, const char* key, int timeout_ms, void* out, size_t cap, size_t* len);
  KvCallbackStore(SetFn set, GetFn get, void* user) : set_(set), get_(get), user_(user) {}
  void set(const std::string& key, const std::vector<char>& data) override;
  std::vector<char> get(const std::string& key, std::chrono::milliseconds timeout) override;

 private:
  SetFn set_;
  GetFn get_;
  void* user_;
};

// Shared directory, one file per key (atomic rename), for ranks that are
// separate processes on one node.
class FileStore : public Store {
 public:
  explicit FileStore(const std::string& dir);
  void set(const std::string& key, const std::vector<char>& data) override;
  std::vector<char> get(const std::string& key, std::chrono::milliseconds timeout) override;

 private:
  std::string path(const std::string& key) const;
  std::string dir_;
};

// In-process store for ranks that are threads of one process.
class HashStore : public Store {
 public:
  void set(const std::string& key, const std::vector<char>& data) override;
  std::vector<char> get(const std::string& key, std::chrono::milliseconds timeout) override;

 private:
  std::mutex m_;
  std::condition_variable cv_;
  std::map<std::string, std::vector<char>> map_;
};

// "file:<dir>" -> FileStore; "mem:<name>" -> a process-wide HashStore shared
// by every caller that names it.
std::shared_ptr<Store> openStore(const std::string& url);

}  // namespace gloo_amd
