// Post-verification analysis kernels (gfx950): K10 k-nearest neighbours for AIF360's
// consistency() and K13 the activation deltas of bias localisation.
//
// fa_knn_kernel<K>   one thread per query row (256 per workgroup), the point set streamed through
//                    LDS in tiles of 128 rows: every lane reads the same point (LDS broadcast),
//                    so the tile costs one conflict-free ds_read per feature.  Squared distances
//                    are summed from exact differences (integer features stay exact in fp32; no
//                    |a|^2 + |b|^2 - 2ab cancellation), the K best are kept sorted in registers
//                    (unrolled insertion, strict comparison: among equal distances the lower
//                    index wins, a deterministic tie rule), the query itself is forced into its
//                    own neighbour set (distance -1), like the device GEMM path of
//                    analysis/metrics.consistency.  Reference: AIF360 consistency (k = 5) called
//                    at src/AC/Verify-AC-experiment-new.py:528.
// fa_actdiff_kernel  one wave64 per counterexample pair (x, x'): both forwards layer by layer,
//                    activations in a wave-private LDS slab, W rows read coalesced across lanes
//                    from global/L2; |act(x) - act(x')| of every neuron (hidden ReLU outputs and
//                    the logit) accumulated in a workgroup LDS array, one global atomic per
//                    neuron per workgroup.  Reference: src/AC/detect_bias.py:223-261 (per-pair
//                    Keras predict of every layer).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "args.h"

#define FA_KNN_TILE 128

template <int K>
__global__ void __launch_bounds__(FA_THREADS) fa_knn_kernel(const float* X, int n, int d, int* idx, float* dist) {
  extern __shared__ float tile[];   // [FA_KNN_TILE][d]
  const int q = blockIdx.x * FA_THREADS + threadIdx.x;
  const bool active = q < n;
  float xq[64];
#pragma unroll
  for (int f = 0; f < 64; ++f) xq[f] = (active && f < d) ? X[(size_t)q * d + f] : 0.f;
  float bd[K];
  int bi[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    bd[i] = INFINITY;
    bi[i] = -1;
  }
  for (int t0 = 0; t0 < n; t0 += FA_KNN_TILE) {
    const int m = min(FA_KNN_TILE, n - t0);
    __syncthreads();
    for (int e = threadIdx.x; e < m * d; e += FA_THREADS) tile[e] = X[(size_t)t0 * d + e];
    __syncthreads();
    if (!active) continue;
    for (int r = 0; r < m; ++r) {
      const float* pt = tile + r * d;
      float s = 0.f;
#pragma unroll
      for (int f = 0; f < 64; ++f) {
        if (f < d) {
          const float df = xq[f] - pt[f];
          s = fmaf(df, df, s);
        }
      }
      const int j = t0 + r;
      if (j == q) s = -1.f;
      if (s < bd[K - 1]) {
        bool placed = false;
#pragma unroll
        for (int i = K - 1; i >= 0; --i) {
          if (!placed) {
            if (i > 0 && bd[i - 1] > s) {
              bd[i] = bd[i - 1];
              bi[i] = bi[i - 1];
            } else {
              bd[i] = s;
              bi[i] = j;
              placed = true;
            }
          }
        }
      }
    }
  }
  if (active) {
#pragma unroll
    for (int i = 0; i < K; ++i) {
      idx[(size_t)q * K + i] = bi[i];
      if (dist) dist[(size_t)q * K + i] = bd[i] < 0.f ? 0.f : bd[i];
    }
  }
}

template <int K>
static int knn_launch_k(const float* X, int n, int d, int* idx, float* dist, hipStream_t stream) {
  const size_t lds = (size_t)FA_KNN_TILE * d * sizeof(float);
  hipLaunchKernelGGL(fa_knn_kernel<K>, dim3((n + FA_THREADS - 1) / FA_THREADS), dim3(FA_THREADS), lds, stream, X, n,
                     d, idx, dist);
  return (int)hipGetLastError();
}

extern "C" int fa_knn_launch(const float* X, int n, int d, int k, int* idx, float* dist, hipStream_t stream) {
  if (n <= 0) return 0;
  if (d <= 0 || d > 64 || k < 1 || k > n) return -3;
  switch (k) {
    case 1: return knn_launch_k<1>(X, n, d, idx, dist, stream);
    case 2: return knn_launch_k<2>(X, n, d, idx, dist, stream);
    case 3: return knn_launch_k<3>(X, n, d, idx, dist, stream);
    case 4: return knn_launch_k<4>(X, n, d, idx, dist, stream);
    case 5: return knn_launch_k<5>(X, n, d, idx, dist, stream);
    case 6: return knn_launch_k<6>(X, n, d, idx, dist, stream);
    case 7: return knn_launch_k<7>(X, n, d, idx, dist, stream);
    case 8: return knn_launch_k<8>(X, n, d, idx, dist, stream);
    case 10: return knn_launch_k<10>(X, n, d, idx, dist, stream);
    case 16: return knn_launch_k<16>(X, n, d, idx, dist, stream);
    default: return -3;
  }
}

// ------------------------------------------------------------------------------------------------
#define FA_AD_WAVES (FA_THREADS / 64)

__global__ void __launch_bounds__(FA_THREADS) fa_actdiff_kernel(NetDesc net, const float* flat, const float* x,
                                                                  const float* xp, int npairs, float* sum_out) {
  extern __shared__ float sm[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int W = net.max_width;
  float* acc = sm;                                  // [n_neurons]
  float* slab = sm + ((net.n_neurons + 3) & ~3) + wave * 4 * W;   // [h, hp, hn, hpn] x W
  for (int j = threadIdx.x; j < net.n_neurons; j += FA_THREADS) acc[j] = 0.f;
  __syncthreads();
  const int n0 = net.dims[0];
  for (int pr = blockIdx.x * FA_AD_WAVES + wave; pr < npairs; pr += gridDim.x * FA_AD_WAVES) {
    float* h = slab;
    float* hp = slab + W;
    float* hn = slab + 2 * W;
    float* hpn = slab + 3 * W;
    for (int i = lane; i < n0; i += 64) {
      h[i] = x[(size_t)pr * n0 + i];
      hp[i] = xp[(size_t)pr * n0 + i];
    }
    __builtin_amdgcn_wave_barrier();
    for (int l = 0; l < net.n_layers; ++l) {
      const int nin = net.dims[l], nout = net.dims[l + 1];
      const float* Wl = flat + net.w_off[l];
      const float* bl = flat + net.b_off[l];
      const bool last = l == net.n_layers - 1;
      for (int j = lane; j < nout; j += 64) {
        float z = bl[j], zp = bl[j];
        for (int i = 0; i < nin; ++i) {
          const float w = Wl[(size_t)i * nout + j];
          z = fmaf(h[i], w, z);
          zp = fmaf(hp[i], w, zp);
        }
        if (!last) {
          z = fmaxf(z, 0.f);
          zp = fmaxf(zp, 0.f);
        }
        hn[j] = z;
        hpn[j] = zp;
        atomicAdd(&acc[net.neuron_off[l] + j], fabsf(z - zp));
      }
      __builtin_amdgcn_wave_barrier();
      float* t = h; h = hn; hn = t;
      t = hp; hp = hpn; hpn = t;
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < net.n_neurons; j += FA_THREADS)
    if (acc[j] != 0.f) atomicAdd(&sum_out[j], acc[j]);
}

extern "C" int fa_actdiff_launch(const NetDesc& net, const float* flat, const float* x, const float* xp, int npairs,
                                 float* sum_out, hipStream_t stream) {
  if (npairs <= 0) return 0;
  const size_t lds = ((size_t)((net.n_neurons + 3) & ~3) + (size_t)FA_AD_WAVES * 4 * net.max_width) * sizeof(float);
  if (lds > 64 * 1024) return -3;
  const int blocks = std::min(1024, (npairs + FA_AD_WAVES - 1) / FA_AD_WAVES);
  hipLaunchKernelGGL(fa_actdiff_kernel, dim3(blocks), dim3(FA_THREADS), lds, stream, net, flat, x, xp, npairs,
                     sum_out);
  return (int)hipGetLastError();
}
