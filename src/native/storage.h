// Pooled host storage manager (see storage.cc).
#pragma once
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace mxamd {

class HostStorage {
 public:
  explicit HostStorage(bool pinned);
  ~HostStorage();
  void* Alloc(size_t size);
  void Free(void* p);
  void ReleaseAll();
  bool pinned() const { return pinned_; }
  size_t used_bytes() const { return used_bytes_; }
  size_t pooled_bytes() const { return pooled_bytes_; }
  uint64_t hits() const { return hits_; }
  uint64_t misses() const { return misses_; }
  static size_t RoundSize(size_t size);

 private:
  void* RawAlloc(size_t size);
  void RawFree(void* p);
  bool pinned_;
  std::mutex mu_;
  std::unordered_map<size_t, std::vector<void*>> free_;
  std::unordered_map<void*, size_t> used_;
  size_t used_bytes_ = 0, pooled_bytes_ = 0;
  uint64_t hits_ = 0, misses_ = 0;
};

}  // namespace mxamd
