// Shared device helpers for the fairify_amd CDNA4 (gfx950) kernels.
//
// Network descriptor, the counter-based RNG shared with ops/reference.py, and the f32 MFMA
// wrapper.  All kernels use 256-thread workgroups = 4 wave64s.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <utility>
#include <vector>

#define FA_MAX_LAYERS 16
#define FA_THREADS 256

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct NetDesc {
  int n_layers;                       // number of weight layers L (last = linear logit)
  int dims[FA_MAX_LAYERS + 1];        // dims[0] = n0 ; dims[l+1] = width of layer l
  int w_off[FA_MAX_LAYERS];           // offset of W_l ([dims[l], dims[l+1]] row-major) in flat
  int b_off[FA_MAX_LAYERS];           // offset of b_l in flat
  int neuron_off[FA_MAX_LAYERS];      // first index of layer l in the all-neuron numbering
  int n_hidden;                       // sum of hidden widths
  int n_neurons;                      // n_hidden + 1
  int max_width;                      // max(dims[0..L])
  int max_wsize;                      // max dims[l]*dims[l+1]
  float unit;                         // unit roundoff of the arithmetic (2^-24)
  float g_gemm[FA_MAX_LAYERS];        // gamma for the layer-l GEMM (K = 2*dims[l] + 1)
  float g_conc;                       // gamma for concretisation sums (K = rows per form)
  float g_one;                        // gamma_1 (interval-row final addition)
  float g_fwd[FA_MAX_LAYERS];         // gamma for the plain forward (K = dims[l] + 1)
  // float offset (multiple of 4) of the MFMA-operand-order copy of the weights in `flat`:
  // per layer [jt][t][lane][i] = W[16t + 4(lane>>4) + i][16jt + (lane&15)] (zero padded), then
  // every layer's bias; staged into LDS by the register-resident kernels with float4 copies
  int wperm_off;
  int wperm_floats;                   // size of that block (multiple of 4)
  // narrow networks (inputs <= 16, hidden layers <= 8 wide): pack_g boxes share one 16-row MFMA
  // tile in the symbolic kernel; block-diagonal weights at pack_off (ops/backend.py:
  // mfma_packed_block), pack_floats long (0 when pack_g == 1)
  int pack_g;
  int pack_off;
  int pack_floats;
  // backward (transposed) operand order of every layer's W, read straight from global memory by
  // the back-substitution kernel when the staged copy would crowd its per-row LDS state out
  // (csrc/refine.hip, BM-4): per layer [ot][t][lane][i] = W[16 ot + (lane&15)][16 t + 4(lane>>4) + i]
  int wback_off;
  int wback_floats;
};

// lowbias32 (Wellons) — identical to ops/reference.py:hash32
__device__ __forceinline__ uint32_t fa_hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

// ops/reference.py:rng_u32 (seed, partition id, sample index, feature index)
__device__ __forceinline__ uint32_t fa_rng(uint32_t seed, int64_t pid, int64_t sample, int dim) {
  uint32_t h = fa_hash32((uint32_t)((uint64_t)(sample * 64 + dim) & 0xFFFFFFFFull) ^ seed);
  h = fa_hash32(h ^ (uint32_t)((uint64_t)pid & 0xFFFFFFFFull));
  h = fa_hash32(h ^ (uint32_t)(((uint64_t)pid >> 32) & 0xFFFFFFFFull) ^ 0x5BD1E995u);
  return h;
}

// One v_mfma_f32_16x16x4_f32: exact f32 fma chain.  Lane l supplies A[l&15][l>>4] and
// B[l>>4][l&15]; D reg i is row (l>>4)*4+i, column l&15.
__device__ __forceinline__ f32x4 fa_mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Compile-time network shape (layer widths dims[0..L]) for kernels specialised to the zoo shapes
// that dominate the workloads (symbolic.hip, refine.hip): layer loops unroll at compile time and
// every width, tile count and lane mask becomes a constant.  FaShapeAny (L = 0): widths from NetDesc.
struct FaShapeAny {
  static constexpr int L = 0;
  __host__ __device__ static constexpr int dim(int) { return 0; }
};
template <int... D>
struct FaShape {
  static constexpr int L = sizeof...(D) - 1;
  __host__ __device__ static constexpr int dim(int i) {
    constexpr int d[] = {D...};
    return d[i];
  }
};

#define FA_CHECK(x)                                                              \
  do {                                                                           \
    hipError_t e__ = (x);                                                        \
    if (e__ != hipSuccess) {                                                     \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e__), __FILE__, \
              __LINE__);                                                         \
      abort();                                                                   \
    }                                                                            \
  } while (0)

// Dynamic-LDS limits.  Every kernel that may be launched with more than 64 KB of dynamic LDS is
// registered at library load by a static initialiser (FA_LDS_REGISTER: pushes the host stub's
// address, no HIP call).  fa_lds_prepare() (csrc/devmem.cpp) raises every registered kernel's limit
// to the device maximum ONCE, when the first Backend is built (ops/backend.py) -- before any host
// thread launches -- so no launch path ever changes a function attribute while other threads
// launch (the round-3 profiled crash had 8 threads racing through per-site hipFuncSetAttribute
// calls).  Launch paths only ask fa_lds_ok(bytes).
inline std::vector<const void*>& fa_lds_registry() {
  static std::vector<const void*> v;
  return v;
}
inline std::atomic<bool>& fa_lds_ready_flag() {
  static std::atomic<bool> ready{false};
  return ready;
}
struct FaLdsReg {
  explicit FaLdsReg(const void* k) { fa_lds_registry().push_back(k); }
};
#define FA_LDS_CAT2(a, b) a##b
#define FA_LDS_CAT(a, b) FA_LDS_CAT2(a, b)
#define FA_LDS_REGISTER(...) \
  static const FaLdsReg FA_LDS_CAT(fa_lds_reg_, __LINE__)[] = {__VA_ARGS__}
#define FA_LDS_K(k) FaLdsReg((const void*)(k))
extern "C" int fa_lds_prepare();
// may a registered kernel be launched with `bytes` of dynamic LDS?
inline bool fa_lds_ok(size_t bytes) { return bytes <= 64 * 1024 || fa_lds_ready_flag().load(std::memory_order_acquire); }
