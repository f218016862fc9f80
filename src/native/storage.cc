// Pooled host storage manager.
//
// Parity: src/storage/pooled_storage_manager.h (GPUPooledStorageManager /
// GPUPooledRoundedStorageManager: size-class free lists, release on OOM),
// pinned_memory_storage.h (cudaHostAlloc) and cpu_device_storage.h.
//
// Device (HBM) memory is owned by the PyTorch caching allocator in this
// framework — one allocator per process keeps the 288 GB of HBM in a single
// pool.  This manager owns the *host* side: page-locked staging buffers for
// host->device copies (data loader batches, checkpoint IO), allocated with
// hipHostMalloc when a HIP runtime and device are present (resolved at run
// time with dlopen so the same .so works on CPU-only hosts) and with
// aligned_alloc otherwise.  Sizes are rounded to power-of-two classes above
// 4 KiB (linear 4 KiB steps below), freed blocks go to per-class free lists.
#include "storage.h"

#include "hip_rt.h"

#include <cstdlib>
#include <cstring>

namespace mxamd {


size_t HostStorage::RoundSize(size_t size) {
  const size_t page = 4096;
  if (size <= page) return page;
  if (size <= (1u << 20)) return (size + page - 1) / page * page;
  size_t r = 1;
  while (r < size) r <<= 1;
  return r;
}

HostStorage::HostStorage(bool pinned) : pinned_(pinned && HipRt::Get().ok) {}

HostStorage::~HostStorage() { ReleaseAll(); }

void* HostStorage::RawAlloc(size_t size) {
  void* p = nullptr;
  if (pinned_) {
    if (HipRt::Get().host_malloc(&p, size, 0) != 0) p = nullptr;
  } else {
    p = std::aligned_alloc(4096, size);
  }
  return p;
}

void HostStorage::RawFree(void* p) {
  if (pinned_)
    HipRt::Get().host_free(p);
  else
    std::free(p);
}

void* HostStorage::Alloc(size_t size) {
  size_t rs = RoundSize(size);
  std::lock_guard<std::mutex> lk(mu_);
  auto it = free_.find(rs);
  void* p = nullptr;
  if (it != free_.end() && !it->second.empty()) {
    p = it->second.back();
    it->second.pop_back();
    pooled_bytes_ -= rs;
    ++hits_;
  } else {
    p = RawAlloc(rs);
    if (!p) {  // out of memory: release the pool and retry once
      for (auto& kv : free_)
        for (void* q : kv.second) RawFree(q);
      free_.clear();
      pooled_bytes_ = 0;
      p = RawAlloc(rs);
      if (!p) return nullptr;
    }
    ++misses_;
  }
  used_[p] = rs;
  used_bytes_ += rs;
  return p;
}

void HostStorage::Free(void* p) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = used_.find(p);
  if (it == used_.end()) return;
  size_t rs = it->second;
  used_.erase(it);
  used_bytes_ -= rs;
  free_[rs].push_back(p);
  pooled_bytes_ += rs;
}

void HostStorage::ReleaseAll() {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& kv : free_)
    for (void* q : kv.second) RawFree(q);
  free_.clear();
  pooled_bytes_ = 0;
}

}  // namespace mxamd
