// Caching device / pinned-host allocators of the native runtimes (see devmem.h).
#include "devmem.h"
#include "common.h"

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace fa_mem {
namespace {

struct Pool {
  std::mutex mu;
  std::map<size_t, std::vector<void*>> free_;    // rounded size -> cached blocks
  std::unordered_map<void*, size_t> live_;        // issued block -> rounded size
  size_t cached_bytes = 0, live_bytes = 0;
  long long mallocs = 0, hits = 0;
};

Pool& dev_pool() {
  static Pool* p = new Pool();    // never destroyed: runtimes may release during interpreter exit
  return *p;
}
Pool& host_pool(bool coherent) {
  static Pool* p0 = new Pool();
  static Pool* p1 = new Pool();
  return coherent ? *p1 : *p0;
}
std::atomic<long long> g_driver_frees{0};
std::mutex g_host_kind_mu;
std::unordered_map<void*, bool> g_host_kind;     // pinned block -> coherent?

void drain(Pool& pool, bool host) {
  for (auto& kv : pool.free_)
    for (void* b : kv.second) {
      if (host) hipHostFree(b);
      else hipFree(b);
      ++g_driver_frees;
    }
  pool.free_.clear();
  pool.cached_bytes = 0;
}

void* take(Pool& pool, size_t bytes) {
  auto it = pool.free_.find(bytes);
  if (it == pool.free_.end() || it->second.empty()) return nullptr;
  void* b = it->second.back();
  it->second.pop_back();
  pool.cached_bytes -= bytes;
  ++pool.hits;
  return b;
}

}  // namespace

size_t round_size(size_t bytes) {
  // classes: multiples of 256 B below 4 KB, then 4 steps per power of two (<= 25 % slack)
  if (bytes <= 4096) return (std::max<size_t>(bytes, 1) + 255) & ~size_t(255);
  int e = 63 - __builtin_clzll((unsigned long long)(bytes - 1));   // 2^e < bytes <= 2^(e+1)
  const size_t step = size_t(1) << (e - 2);
  return (bytes + step - 1) / step * step;
}

void* dev_alloc(size_t bytes) {
  bytes = round_size(bytes);
  Pool& pool = dev_pool();
  std::lock_guard<std::mutex> g(pool.mu);
  void* b = take(pool, bytes);
  if (!b) {
    hipError_t e = hipMalloc(&b, bytes);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      hipDeviceSynchronize();
      drain(pool, false);
      e = hipMalloc(&b, bytes);
    }
    if (e != hipSuccess) throw std::runtime_error(std::string("hipMalloc: ") + hipGetErrorString(e));
    ++pool.mallocs;
  }
  pool.live_[b] = bytes;
  pool.live_bytes += bytes;
  return b;
}

void dev_release(void* p) {
  if (!p) return;
  Pool& pool = dev_pool();
  std::lock_guard<std::mutex> g(pool.mu);
  auto it = pool.live_.find(p);
  if (it == pool.live_.end()) return;            // not ours: never free foreign pointers
  const size_t bytes = it->second;
  pool.live_.erase(it);
  pool.live_bytes -= bytes;
  pool.free_[bytes].push_back(p);
  pool.cached_bytes += bytes;
}

void* host_alloc(size_t bytes, bool coherent) {
  bytes = round_size(bytes);
  Pool& pool = host_pool(coherent);
  void* b = nullptr;
  {
    std::lock_guard<std::mutex> g(pool.mu);
    b = take(pool, bytes);
    if (!b) {
      hipError_t e = hipHostMalloc(&b, bytes, coherent ? hipHostMallocCoherent : hipHostMallocDefault);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        hipDeviceSynchronize();
        drain(pool, true);
        e = hipHostMalloc(&b, bytes, coherent ? hipHostMallocCoherent : hipHostMallocDefault);
      }
      if (e != hipSuccess) throw std::runtime_error(std::string("hipHostMalloc: ") + hipGetErrorString(e));
      ++pool.mallocs;
    }
    pool.live_[b] = bytes;
    pool.live_bytes += bytes;
  }
  std::lock_guard<std::mutex> g(g_host_kind_mu);
  g_host_kind[b] = coherent;
  return b;
}

void host_release(void* p) {
  if (!p) return;
  bool coherent;
  {
    std::lock_guard<std::mutex> g(g_host_kind_mu);
    auto k = g_host_kind.find(p);
    if (k == g_host_kind.end()) return;
    coherent = k->second;
  }
  Pool& pool = host_pool(coherent);
  std::lock_guard<std::mutex> g(pool.mu);
  auto it = pool.live_.find(p);
  if (it == pool.live_.end()) return;
  const size_t bytes = it->second;
  pool.live_.erase(it);
  pool.live_bytes -= bytes;
  pool.free_[bytes].push_back(p);
  pool.cached_bytes += bytes;
}

Stats stats() {
  Stats s{};
  {
    Pool& d = dev_pool();
    std::lock_guard<std::mutex> g(d.mu);
    s.dev_cached_bytes = d.cached_bytes;
    s.dev_live_bytes = d.live_bytes;
    s.dev_mallocs = d.mallocs;
    s.dev_hits = d.hits;
  }
  for (bool coh : {false, true}) {
    Pool& h = host_pool(coh);
    std::lock_guard<std::mutex> g(h.mu);
    s.host_cached_bytes += h.cached_bytes;
    s.host_live_bytes += h.live_bytes;
    s.host_mallocs += h.mallocs;
    s.host_hits += h.hits;
  }
  s.driver_frees = g_driver_frees.load();
  return s;
}

void release_cached() {
  hipDeviceSynchronize();
  {
    Pool& d = dev_pool();
    std::lock_guard<std::mutex> g(d.mu);
    drain(d, false);
  }
  for (bool coh : {false, true}) {
    Pool& h = host_pool(coh);
    std::lock_guard<std::mutex> g(h.mu);
    drain(h, true);
  }
}

}  // namespace fa_mem

// ------------------------------------------------------------------------------------------------
// Dynamic-LDS registry (common.h): raise every registered kernel's limit to the device maximum
// once.  Called from Backend construction (bindings: prepare_lds) before host threads launch;
// magic-static initialisation makes concurrent first calls wait for the one that runs.
extern "C" int fa_lds_prepare() {
  static const int rc = [] {
    int dev = 0, maxb = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    if (hipDeviceGetAttribute(&maxb, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess || maxb <= 0)
      maxb = 160 * 1024;
    for (const void* k : fa_lds_registry()) {
      hipFuncAttributes at{};
      if (hipFuncGetAttributes(&at, k) != hipSuccess) return -2;
      const int dyn = maxb - (int)at.sharedSizeBytes;
      if (dyn <= 64 * 1024) continue;
      if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, dyn) != hipSuccess) return -3;
    }
    fa_lds_ready_flag().store(true, std::memory_order_release);
    return 0;
  }();
  return rc;
}
