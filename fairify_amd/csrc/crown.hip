// Backward (CROWN-style) output bounds on top of the forward symbolic pass (K4 refinement).
// gfx950.  Same arithmetic and error terms as ops/reference.py:crown_output.
//
// The forward kernels (symbolic.hip / bounds.hip) concretise every layer's linear forms before
// relaxing its ReLUs, so each layer's relaxation slack travels forward as a fixed interval.
// Here one wave64 per box-row back-substitutes the logit through the network instead: the
// multiplier lambda_j of neuron j picks the relaxation its sign needs (lambda >= 0: h >= a z,
// a in {0, 1}; lambda < 0: the chord h <= s (z - l)), using the per-neuron pre-activation
// bounds the forward pass wrote (layer_lb / layer_ub) as relaxation intervals.  Lower and upper
// bounds are two multiplier vectors processed together.  On the deep AC shapes this halves the
// open branch-and-bound frontier (tools/diag_open_nodes.py --bound crown).
//
// Layout: the row-major weights + biases (the `flat` prefix [W_0|b_0|W_1|b_1|...]) are staged
// once per workgroup in LDS; each wave owns a slab [lambda(2) | mu(2)] x FA_CROWN_MAXW.  Per
// layer: lanes over the layer's neurons form mu = lambda * slope (+ chord intercepts), then
// lanes over the layer's inputs form lambda' = W mu (and |W| |mu| for the rounding term).
// The wave writes the back-substituted forms where they concretise tighter than the forward
// ones and intersects the logit bounds.
//
// Rounding: only chord multipliers/intercepts, the W mu dot products and the constant sums are
// rounded; each carries a gamma-bounded error weighted by the magnitude of the quantity it
// multiplies (|z| <= max(|l|, |u|), |h| <= max(0, u), |x| on the box), accumulated into the
// form's error term -- so sigma * y >= lambda . x + c - err holds for the exact network.
#include <hip/hip_runtime.h>

#include <mutex>

#include "args.h"

#define FA_CROWN_MAXW 256
#define FA_CROWN_WAVES 4

__device__ __forceinline__ float fa_gam(int k, float u) {
  const float ku = (float)(k + 2) * u;
  return ku / (1.f - ku) * (1.f + 4.f * u);
}

__device__ __forceinline__ float fa_wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__global__ void __launch_bounds__(64 * FA_CROWN_WAVES) fa_crown_kernel(NetDesc net, BoundArgs a, int nparams) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  for (int e = tid; e < nparams; e += 64 * FA_CROWN_WAVES) smem[e] = a.flat[e];
  __syncthreads();
  const int lane = tid & 63;
  const int wave = tid >> 6;
  float* lam = smem + nparams + wave * 4 * FA_CROWN_MAXW;   // [2][MAXW]
  float* mu = lam + 2 * FA_CROWN_MAXW;                     // [2][MAXW]
  const int L = net.n_layers;
  const int n0 = net.dims[0];
  const int N = net.n_neurons;
  const float u = net.unit;
  for (int r0 = blockIdx.x * FA_CROWN_WAVES + wave; r0 < a.R; r0 += gridDim.x * FA_CROWN_WAVES) {
    const int r = __builtin_amdgcn_readfirstlane(r0);
    const int node = a.V > 0 ? r / a.V : r;
    const int v = a.V > 0 ? r - node * a.V : 0;
    const uint8_t* dmask = nullptr;             // forced-dead hidden neurons of this row
    if (a.dead_in) dmask = a.dead_in + (size_t)r * net.n_hidden;
    else if (a.dead_part) dmask = a.dead_part + (size_t)a.node_part[node] * net.n_hidden;
    const float* lbr = a.layer_lb + (size_t)r * N;
    const float* ubr = a.layer_ub + (size_t)r * N;
    // ---- init: lambda = +-W_{L-1}[:, 0], c = +-b_{L-1}
    {
      const int n = net.dims[L - 1];
      const float* W = smem + net.w_off[L - 1];
      for (int i = lane; i < n; i += 64) {
        lam[i] = W[i];
        lam[FA_CROWN_MAXW + i] = -W[i];
      }
    }
    float c[2], err[2];
    c[0] = smem[net.b_off[L - 1]];
    c[1] = -c[0];
    err[0] = err[1] = 0.f;
    __builtin_amdgcn_wave_barrier();
    for (int l = L - 2; l >= 0; --l) {
      const int n = net.dims[l + 1];
      const int nin = net.dims[l];
      const int off = net.neuron_off[l];
      const float* W = smem + net.w_off[l];
      const float* b = smem + net.b_off[l];
      float cs[2] = {0.f, 0.f}, cm[2] = {0.f, 0.f}, er[2] = {0.f, 0.f};
      for (int j = lane; j < n; j += 64) {
        const float lb = lbr[off + j], ub = ubr[off + j];
        const bool dd = ub <= 0.f || (dmask && dmask[off + j]);
        const bool act = !dd && lb >= 0.f;
        const bool unst = !dd && !act;
        const float alpha = ub > -lb ? 1.f : 0.f;
        const float s = unst ? (ub / (ub - lb)) * (1.f + 4.f * u) : 0.f;
        const float zmax = fmaxf(fabsf(lb), fabsf(ub));
        const float bj = b[j];
#pragma unroll
        for (int sg = 0; sg < 2; ++sg) {
          const float lm = lam[sg * FA_CROWN_MAXW + j];
          const float slope = act ? 1.f : (dd ? 0.f : (lm >= 0.f ? alpha : s));
          const float m = lm * slope;
          const bool neg = unst && lm < 0.f;
          const float t = neg ? -m * lb : 0.f;
          mu[sg * FA_CROWN_MAXW + j] = m;
          cs[sg] += m * bj + t;
          cm[sg] += fabsf(m * bj) + fabsf(t);
          if (neg) er[sg] += 3.f * u * (fabsf(m) * zmax + fabsf(t));
        }
      }
      __builtin_amdgcn_wave_barrier();
      const float gn = fa_gam(n + 1, u);
      for (int i = lane; i < nin; i += 64) {
        float acc0 = 0.f, acc1 = 0.f, mag0 = 0.f, mag1 = 0.f;
        const float* Wi = W + (size_t)i * n;
        for (int j = 0; j < n; ++j) {
          const float w = Wi[j];
          const float m0 = mu[j], m1 = mu[FA_CROWN_MAXW + j];
          acc0 = fmaf(w, m0, acc0);
          acc1 = fmaf(w, m1, acc1);
          mag0 = fmaf(fabsf(w), fabsf(m0), mag0);
          mag1 = fmaf(fabsf(w), fabsf(m1), mag1);
        }
        float hm;
        if (l > 0) {
          const int po = net.neuron_off[l - 1];
          hm = fmaxf(ubr[po + i], 0.f);
          if (dmask && dmask[po + i]) hm = 0.f;
        } else {
          float xl = a.lo[(size_t)node * n0 + i], xh = a.hi[(size_t)node * n0 + i];
          if (a.V > 0)
            for (int k = 0; k < a.npa; ++k)
              if (a.pa_idx[k] == i) xl = xh = a.values[v * a.npa + k];
          hm = fmaxf(fabsf(xl), fabsf(xh));
        }
        lam[i] = acc0;
        lam[FA_CROWN_MAXW + i] = acc1;
        er[0] += gn * mag0 * hm;
        er[1] += gn * mag1 * hm;
      }
      const float gc = fa_gam(2 * n + 1, u);
#pragma unroll
      for (int sg = 0; sg < 2; ++sg) {
        const float csum = fa_wave_sum(cs[sg]);
        const float cmag = fa_wave_sum(cm[sg]);
        const float esum = fa_wave_sum(er[sg]);
        const float cold = c[sg];
        c[sg] = cold + csum;
        err[sg] += esum + gc * (fabsf(cold) + cmag);
      }
      __builtin_amdgcn_wave_barrier();
    }
    // ---- concretise over the input box
    int K = 4 * L + 4;
    for (int l = 0; l < L; ++l) K += 2 * net.dims[l + 1];
    const float gK = fa_gam(K, u);
    const float g0 = fa_gam(n0 + 1, u);
    const float g1 = fa_gam(1, u);
    float low[2];
#pragma unroll
    for (int sg = 0; sg < 2; ++sg) {
      float cp = 0.f, mp = 0.f;
      for (int i = lane; i < n0; i += 64) {
        float xl = a.lo[(size_t)node * n0 + i], xh = a.hi[(size_t)node * n0 + i];
        if (a.V > 0)
          for (int k = 0; k < a.npa; ++k)
            if (a.pa_idx[k] == i) xl = xh = a.values[v * a.npa + k];
        const float lm = lam[sg * FA_CROWN_MAXW + i];
        cp += fminf(lm * xl, lm * xh);
        mp += fabsf(lm) * fmaxf(fabsf(xl), fabsf(xh));
      }
      const float conc = fa_wave_sum(cp) + c[sg];
      const float cmg = fa_wave_sum(mp) + fabsf(c[sg]);
      err[sg] *= 1.f + 2.f * gK;
      low[sg] = conc - err[sg] - g0 * cmg - g1 * fabsf(conc);
    }
    const float olb = a.out_lb[r], oub = a.out_ub[r];
    const bool useL = low[0] >= olb;
    const bool useU = -low[1] <= oub;
    for (int i = lane; i < n0; i += 64) {
      if (useL) a.Lc[(size_t)r * n0 + i] = lam[i];
      if (useU) a.Uc[(size_t)r * n0 + i] = -lam[FA_CROWN_MAXW + i];
    }
    if (lane == 0) {
      if (useL) { a.L0[r] = c[0]; a.Le[r] = err[0]; a.out_lb[r] = low[0]; }
      if (useU) { a.U0[r] = -c[1]; a.Ue[r] = err[1]; a.out_ub[r] = -low[1]; }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// 0 on success; -1 if the network does not fit (a layer wider than FA_CROWN_MAXW or weights
// beyond the LDS budget) -- callers then keep the forward forms.
extern "C" int fa_crown_launch(const NetDesc& net, BoundArgs a, hipStream_t stream) {
  if (a.R <= 0) return 0;
  if (!a.layer_lb || !a.layer_ub || !a.Lc || !a.Uc) return -2;
  for (int l = 0; l <= net.n_layers; ++l)
    if (net.dims[l] > FA_CROWN_MAXW) return -1;
  int nparams = 0;
  for (int l = 0; l < net.n_layers; ++l) nparams = net.b_off[l] + net.dims[l + 1];
  const size_t bytes = ((size_t)nparams + (size_t)FA_CROWN_WAVES * 4 * FA_CROWN_MAXW) * sizeof(float);
  if (bytes > 160 * 1024) return -1;
  static std::mutex mu;
  static size_t raised = 0;
  if (bytes > 64 * 1024) {
    std::lock_guard<std::mutex> g(mu);
    if (bytes > raised) {
      if (hipFuncSetAttribute((const void*)fa_crown_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) !=
          hipSuccess)
        return -3;
      raised = bytes;
    }
  }
  const int blocks = (int)std::min<long long>(((long long)a.R + FA_CROWN_WAVES - 1) / FA_CROWN_WAVES, 256LL * 8);
  hipLaunchKernelGGL(fa_crown_kernel, dim3(blocks), dim3(64 * FA_CROWN_WAVES), bytes, stream, net, a, nparams);
  return (int)hipGetLastError();
}
