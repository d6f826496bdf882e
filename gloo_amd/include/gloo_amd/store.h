// store.h — rendezvous key/value stores (mirrors gloo::rendezvous::Store,
// gloo/rendezvous/store.h, FileStore gloo/rendezvous/file_store.h:19 and
// HashStore gloo/rendezvous/hash_store.h:20).  Used only at setup: to publish
// each rank's inbox arena (IPC handle) and the control block's name.
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
