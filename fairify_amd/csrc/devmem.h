// Process-wide caching allocators for the native runtimes' device and pinned host buffers.
//
// hipFree and hipHostFree synchronise the whole device and hold the runtime's allocation lock
// while they wait: every other host thread's kernel launches and copies block behind them.  On
// the 1/8-shard bench, buffer regrowth (free + malloc of a slightly larger block) inside the
// timed steps issued ~180 hipFree per 3 steps, one of them stalling all 8 host threads for
// 21 ms with the GPU idle (rocprofv3 --hip-trace, profiles/r3/emu/gaps.txt).  Blocks released
// here go to a free list keyed by their rounded size and are handed out again; nothing is
// returned to the driver until an allocation fails (then the device is synchronised once, the
// cache released, and the allocation retried) or the process exits.
//
// Stream safety: a block may be re-issued to ANOTHER runtime / stream as soon as it is released,
// so release only blocks no queued GPU work still touches.  The runtimes release at two kinds of
// points, both after a hipStreamSynchronize of the only stream that used the block: buffer
// regrowth (solve start, after the previous solve's final sync; level start, after the level-end
// sync) and runtime destruction (after its last solve returned).  The buffer-lifetime rule of
// tests/test_stream_lifetime.py covers the pinned host side the same way.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <stdexcept>
#include <string>

namespace fa_mem {

void* dev_alloc(size_t bytes);             // >= bytes, device memory
void dev_release(void* p);                 // back to the cache (nullptr: no-op)
void* host_alloc(size_t bytes, bool coherent);   // >= bytes, pinned (hipHostMalloc)
void host_release(void* p);
size_t round_size(size_t bytes);           // the size class a request is served from

struct Stats {
  size_t dev_cached_bytes, dev_live_bytes, host_cached_bytes, host_live_bytes;
  long long dev_mallocs, dev_hits, host_mallocs, host_hits, driver_frees;
};
Stats stats();
void release_cached();                     // synchronise the device, give every cached block back

// Device buffer of T that grows (never shrinks) through the cache; contents are NOT preserved on
// growth.  Growth requests are rounded up to the cache's size classes.
template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  void ensure(size_t cnt) {
    if (cnt <= n) return;
    dev_release(p);
    p = nullptr;
    const size_t bytes = round_size(std::max<size_t>(cnt, 1) * sizeof(T));
    p = static_cast<T*>(dev_alloc(bytes));
    n = bytes / sizeof(T);
  }
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { dev_release(p); }
};

// Pinned host staging block (bytes), grown through the cache.
struct HostBuf {
  unsigned char* p = nullptr;
  size_t n = 0;
  bool coherent = false;
  void ensure(size_t need) {
    if (need <= n) return;
    host_release(p);
    p = nullptr;
    const size_t bytes = round_size(std::max(std::max<size_t>(need, 4096), 2 * n));
    p = static_cast<unsigned char*>(host_alloc(bytes, coherent));
    n = bytes;
  }
  HostBuf() = default;
  explicit HostBuf(bool coh) : coherent(coh) {}
  HostBuf(const HostBuf&) = delete;
  HostBuf& operator=(const HostBuf&) = delete;
  ~HostBuf() { host_release(p); }
};

}  // namespace fa_mem
