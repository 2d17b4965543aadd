// Rigorous point evaluation: logit + running fp32 error bound at integer points.  gfx950.
//
// Used by the branch-and-bound runtime to screen candidate counterexample pairs (every BFS
// level evaluates the LP-optimal vertex pair of every open node) and by the tensor BaB.  It
// replaces interval bound propagation on degenerate boxes (the reference replays candidate
// points with plain `net`, src/AC/Verify-AC.py:229-254; its soundness comes from Z3).
//
// Per layer, with h the fp32 inputs and e a bound on |h_exact - h|:
//     z = W^T h + b                                   (MFMA fma chain, one rounding per product)
//     d = (|W|^T (e + g|h|)) (1 + 2g) + g|b| + g1|z|  (g = gamma(K) of the GEMM, g1 = gamma(1))
// so |v_exact - z| <= d.  ReLU is 1-Lipschitz: h' = max(z, 0), e' = d — except that a neuron
// with z + d <= 0 (or forced dead) is exactly 0 with e' = 0, which keeps the exact zeros of
// sign-structured sums exact.  Output: [z - d, z + d].
//
// Layout (same as the symbolic kernel, csrc/symbolic.hip): one wave64 owns 16 points = the 16
// columns of v_mfma_f32_16x16x4_f32 tiles whose rows are neurons; the accumulator tile of layer
// l is the B operand of layer l+1 (reg i of tile t = neuron 16t + 4*(lane>>4) + i), W is staged
// once per workgroup in LDS in MFMA operand order.  Two products per K step: W.h and
// |W|.(e + g|h|); the epilogue is purely elementwise (no cross-lane traffic).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <mutex>

#include "args.h"

struct PointCfg {
  int w_lds[FA_MAX_LAYERS];   // LDS float offset of W_l in MFMA operand order
  int b_lds[FA_MAX_LAYERS];
};

template <int TM>
__device__ __forceinline__ void fa_point_layer(const NetDesc& net, const BoundArgs& a, const PointCfg& cfg,
                                               const float* smem, int l, int p0, int lane,
                                               const float (&H)[TM][4], const float (&E)[TM][4],
                                               float (&H2)[TM][4], float (&E2)[TM][4]) {
  const int col = lane & 15, grp = lane >> 4;
  const int n_in = net.dims[l], n_out = net.dims[l + 1];
  const int tin = (n_in + 15) >> 4, tout = (n_out + 15) >> 4;
  const float* sw = smem + cfg.w_lds[l];
  const float* sb = smem + cfg.b_lds[l];
  const bool last = l == net.n_layers - 1;
  const float gg = net.g_fwd[l];
  const float gi = net.g_one;
  const float gnext = last ? 0.f : net.g_fwd[l + 1];
  const int noff = net.neuron_off[l];
  const int p = p0 + col;
  const bool pv = p < a.R;
#pragma unroll
  for (int jt = 0; jt < TM; ++jt) {
    if (jt >= tout) break;
    f32x4 Z = {0.f, 0.f, 0.f, 0.f}, Q = {0.f, 0.f, 0.f, 0.f};
    const float4* wq = reinterpret_cast<const float4*>(sw) + (size_t)jt * tin * 64 + lane;
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      if (t >= tin) break;
      const float4 w4 = wq[t * 64];
      const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        Z = fa_mfma4(wv[i], H[t][i], Z);
        Q = fa_mfma4(fabsf(wv[i]), E[t][i], Q);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = 16 * jt + 4 * grp + i;
      const bool jv = j < n_out;
      const float b = jv ? sb[j] : 0.f;
      const float z = Z[i] + b;
      const float d = Q[i] * (1.f + 2.f * gg) + gg * fabsf(b) + gi * fabsf(z);
      if (last) {
        if (j == 0 && pv) {
          a.out_lb[p] = z - d;
          a.out_ub[p] = z + d;
        }
        continue;
      }
      bool forced = false;
      if (jv && pv) {
        if (a.dead_in) forced = a.dead_in[(size_t)p * net.n_hidden + noff + j] != 0;
        else if (a.dead_part)
          forced = a.dead_part[(size_t)a.node_part[a.part_mod ? p % a.part_mod : p] * net.n_hidden + noff + j] != 0;
      }
      const bool zero = !jv || forced || (z + d <= 0.f);
      const float h = zero ? 0.f : fmaxf(z, 0.f);
      const float e = zero ? 0.f : d;
      H2[jt][i] = h;
      E2[jt][i] = e + gnext * h;       // next layer's error operand: e + g |h|  (h >= 0)
    }
  }
}

// 7-tile nets: 260 -> 254 VGPRs (spill-free) doubles the waves per SIMD (1 -> 2)
template <int TM>
__global__ void __launch_bounds__(FA_THREADS) __attribute__((amdgpu_waves_per_eu(TM == 7 ? 2 : 1))) fa_point_kernel(NetDesc net, BoundArgs a, PointCfg cfg) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  // ---- stage the MFMA-operand-order weights + biases (pre-permuted in `flat`) into LDS
  {
    const float4* src = reinterpret_cast<const float4*>(a.flat + net.wperm_off);
    float4* dst = reinterpret_cast<float4*>(smem);
    for (int e = tid; e < (net.wperm_floats >> 2); e += FA_THREADS) dst[e] = src[e];
  }
  __syncthreads();
  const int lane = tid & 63, col = lane & 15, grp = lane >> 4;
  const int wave = tid >> 6, nw = FA_THREADS / 64;
  const int n0 = net.dims[0];
  const int tin0 = (n0 + 15) >> 4;
  const float g0 = net.g_fwd[0];
  const int ntile = (a.R + 15) >> 4;
  for (int tile = blockIdx.x * nw + wave; tile < ntile; tile += gridDim.x * nw) {
    const int p0 = tile * 16;
    const int p = p0 + col;
    if (a.row_open && !__any(p < a.R && a.row_open[p % a.open_mod])) continue;   // wave-uniform
    float HA[TM][4], EA[TM][4], HB[TM][4], EB[TM][4];
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      if (t >= tin0) break;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = 16 * t + 4 * grp + i;
        const float x = (k < n0 && p < a.R) ? a.lo[(size_t)p * n0 + k] : 0.f;
        HA[t][i] = x;
        EA[t][i] = g0 * fabsf(x);      // inputs are exact: only the GEMM rounding term
      }
    }
    for (int l = 0; l < net.n_layers; ++l) {
      if (l & 1) fa_point_layer<TM>(net, a, cfg, smem, l, p0, lane, HB, EB, HA, EA);
      else fa_point_layer<TM>(net, a, cfg, smem, l, p0, lane, HA, EA, HB, EB);
    }
  }
}

namespace {
typedef void (*PointKernel)(NetDesc, BoundArgs, PointCfg);

PointKernel select_point(int TM) {
  if (TM <= 1) return fa_point_kernel<1>;
  if (TM <= 2) return fa_point_kernel<2>;
  if (TM <= 4) return fa_point_kernel<4>;
  if (TM <= 7) return fa_point_kernel<7>;
  // BM-4's 150-wide layer: the unroller gives up on the 10x10-tile body and the operand arrays
  // live in scratch (656 B/lane), still far cheaper than the IBP fallback, which stages each
  // layer's W per box row (one 90 KB row per workgroup: G = 1)
  if (TM <= 10) return fa_point_kernel<10>;
  return nullptr;   // wider layers: the caller falls back to IBP
}

int point_cus() {
  static int cus = 0;
  static std::once_flag once;
  std::call_once(once, [] {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  });
  return cus;
}
}  // namespace

// Rigorous point forward over a.R points a.lo [R, n0] (a.hi ignored); writes a.out_lb/out_ub.
// Honours a.dead_in (per point) or a.dead_part + a.node_part (per point's partition).
// Returns 1 if launched, 0 if the shape is unsupported (caller falls back), <0 on error.
extern "C" int fa_point_try_launch(const NetDesc& net, BoundArgs a, hipStream_t stream) {
  if (a.R <= 0) return 1;
  int TM = 1;
  for (int l = 0; l <= net.n_layers; ++l) TM = std::max(TM, (net.dims[l] + 15) / 16);
  PointKernel k = select_point(TM);
  if (!k) return 0;
  PointCfg cfg{};
  int off = 0;
  for (int l = 0; l < net.n_layers; ++l) {
    cfg.w_lds[l] = off;
    off += ((net.dims[l] + 15) / 16) * ((net.dims[l + 1] + 15) / 16) * 256;
  }
  for (int l = 0; l < net.n_layers; ++l) {
    cfg.b_lds[l] = off;
    off += net.dims[l + 1];
  }
  if (((off + 3) & ~3) != net.wperm_floats) return -1;   // layout mismatch with the pre-permuted block
  const size_t bytes = (size_t)((off + 3) & ~3) * sizeof(float);
  if (bytes > 150 * 1024) return 0;
  static std::mutex mu;
  static std::map<std::pair<const void*, size_t>, int> occ;
  int per_cu = 0;
  {
    std::lock_guard<std::mutex> g(mu);
    const auto key = std::make_pair((const void*)k, bytes);
    auto it = occ.find(key);
    if (it == occ.end()) {
      if (!fa_lds_ok(bytes)) return -4;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, FA_THREADS, bytes) != hipSuccess || per_cu <= 0)
        per_cu = 1;
      occ[key] = per_cu;
    } else {
      per_cu = it->second;
    }
  }
  const long long tiles = (a.R + 15) / 16;
  long long blocks = (tiles + 3) / 4;
  const long long cap = (long long)point_cus() * per_cu;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(FA_THREADS), bytes, stream, net, a, cfg);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 1 : -(int)e;
}

FA_LDS_REGISTER(FA_LDS_K(fa_point_kernel<1>), FA_LDS_K(fa_point_kernel<2>), FA_LDS_K(fa_point_kernel<4>),
                FA_LDS_K(fa_point_kernel<7>), FA_LDS_K(fa_point_kernel<10>));
