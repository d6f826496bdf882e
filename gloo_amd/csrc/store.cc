// store.cc — FileStore / HashStore (see store.h).
#include "gloo_amd/store.h"

#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <thread>

#include "gloo_amd/common.h"

namespace gloo_amd {

FileStore::FileStore(const std::string& dir) : dir_(dir) {
  ::mkdir(dir_.c_str(), 0777);  // may already exist
}

std::string FileStore::path(const std::string& key) const {
  std::string k;
  for (char c : key) k += (c == '/') ? '%' : c;
  return dir_ + "/" + k;
}

void FileStore::set(const std::string& key, const std::vector<char>& data) {
  const std::string final_path = path(key);
  const std::string tmp = final_path + ".tmp." + std::to_string(::getpid()) + "." +
                          std::to_string(std::hash<std::thread::id>()(std::this_thread::get_id()));
  {
    std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
    GLOO_AMD_ENFORCE(f.good(), "cannot write ", tmp);
    f.write(data.data(), (std::streamsize)data.size());
  }
  GLOO_AMD_ENFORCE(::rename(tmp.c_str(), final_path.c_str()) == 0, "rename failed for ", final_path);
}

std::vector<char> FileStore::get(const std::string& key, std::chrono::milliseconds timeout) {
  const std::string p = path(key);
  const auto deadline = std::chrono::steady_clock::now() + timeout;
  auto sleep = std::chrono::microseconds(50);
  for (;;) {
    std::ifstream f(p, std::ios::binary);
    if (f.good()) return std::vector<char>(std::istreambuf_iterator<char>(f), {});
    if (std::chrono::steady_clock::now() > deadline)
      throw IoException("FileStore: timed out waiting for key " + key);
    std::this_thread::sleep_for(sleep);
    if (sleep < std::chrono::milliseconds(5)) sleep *= 2;
  }
}

void HashStore::set(const std::string& key, const std::vector<char>& data) {
  std::lock_guard<std::mutex> lk(m_);
  map_[key] = data;
  cv_.notify_all();
}

std::vector<char> HashStore::get(const std::string& key, std::chrono::milliseconds timeout) {
  std::unique_lock<std::mutex> lk(m_);
  if (!cv_.wait_for(lk, timeout, [&] { return map_.count(key) > 0; }))
    throw IoException("HashStore: timed out waiting for key " + key);
  return map_[key];
}

std::vector<std::vector<char>> Store::allgather(const std::string& tag, int rank, int size,
                                               const std::vector<char>& mine, std::chrono::milliseconds timeout) {
  set(tag + "/" + std::to_string(rank), mine);
  std::vector<std::vector<char>> all(size);
  for (int r = 0; r < size; r++) all[r] = r == rank ? mine : get(tag + "/" + std::to_string(r), timeout);
  return all;
}

void CallbackStore::set(const std::string&, const std::vector<char>&) {
  throw EnforceNotMet("CallbackStore supports only collective all-gathers");
}

std::vector<char> CallbackStore::get(const std::string&, std::chrono::milliseconds) {
  throw EnforceNotMet("CallbackStore supports only collective all-gathers");
}

std::vector<std::vector<char>> CallbackStore::allgather(const std::string& tag, int, int size,
                                                       const std::vector<char>& mine, std::chrono::milliseconds) {
  GLOO_AMD_ENFORCE(mine.size() + 4 <= kBlock, "bootstrap record of ", mine.size(), " bytes exceeds the block");
  std::vector<char> in(kBlock, 0), out(kBlock * (size_t)size, 0);
  const uint32_t len = (uint32_t)mine.size();
  std::memcpy(in.data(), &len, 4);
  if (len) std::memcpy(in.data() + 4, mine.data(), len);
  if (fn_(user_, in.data(), out.data(), kBlock) != 0)
    throw IoException("bootstrap all-gather failed (" + tag + ")");
  std::vector<std::vector<char>> all(size);
  for (int r = 0; r < size; r++) {
    uint32_t l = 0;
    std::memcpy(&l, out.data() + (size_t)r * kBlock, 4);
    GLOO_AMD_ENFORCE(l + 4 <= kBlock, "bad bootstrap block from rank ", r);
    all[r].assign(out.data() + (size_t)r * kBlock + 4, out.data() + (size_t)r * kBlock + 4 + l);
  }
  return all;
}

void KvCallbackStore::set(const std::string& key, const std::vector<char>& data) {
  if (set_(user_, key.c_str(), data.data(), data.size()) != 0) throw IoException("store set failed: " + key);
}

std::vector<char> KvCallbackStore::get(const std::string& key, std::chrono::milliseconds timeout) {
  std::vector<char> v(256);
  for (int attempt = 0; attempt < 2; attempt++) {
    size_t len = 0;
    const int rc = get_(user_, key.c_str(), (int)timeout.count(), v.data(), v.size(), &len);
    if (rc != 0) throw IoException(strcat_("store get of ", key, " failed or timed out after ", timeout.count(), " ms"));
    if (len <= v.size()) {
      v.resize(len);
      return v;
    }
    v.resize(len);  // the value is longer than the buffer: fetch it again in full
  }
  throw EnforceNotMet("store value of " + key + " changed size between two gets");
}

std::shared_ptr<Store> openStore(const std::string& url) {
  static std::mutex m;
  static std::map<std::string, std::weak_ptr<Store>> named;
  if (url.rfind("file:", 0) == 0) return std::make_shared<FileStore>(url.substr(5));
  if (url.rfind("mem:", 0) == 0) {
    std::lock_guard<std::mutex> lk(m);
    auto sp = named[url].lock();
    if (!sp) {
      sp = std::make_shared<HashStore>();
      named[url] = sp;
    }
    return sp;
  }
  throw EnforceNotMet("unknown store url (want file:<dir> or mem:<name>): " + url);
}

}  // namespace gloo_amd
