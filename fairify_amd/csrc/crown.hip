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
// Layout: the weights + biases (the `flat` prefix [W_0|b_0|W_1|b_1|...], each W_l transposed to
// [n_out][n_in]) are staged once per workgroup in LDS; a group of G lanes (G = widest layer rounded up to a power of two,
// 4..64) owns a row and a slab [lambda(2) | mu(2)] x WP.  Per layer: lanes over the layer's
// neurons form mu = lambda * slope (+ chord intercepts), then lanes over the layer's inputs
// form lambda' = W mu (and |W| |mu| for the rounding term).
// The wave writes the back-substituted forms where they concretise tighter than the forward
// ones and intersects the logit bounds.
//
// Rounding: only chord multipliers/intercepts, the W mu dot products and the constant sums are
// rounded; each carries a gamma-bounded error weighted by the magnitude of the quantity it
// multiplies (|z| <= max(|l|, |u|), |h| <= max(0, u), |x| on the box), accumulated into the
// form's error term -- so sigma * y >= lambda . x + c - err holds for the exact network.
#include <hip/hip_runtime.h>

#include <stdlib.h>

#include <algorithm>
#include <map>
#include <mutex>

#include "args.h"

#define FA_CROWN_MAXW 256
#define FA_CROWN_WAVES 4

__device__ __forceinline__ float fa_gam(int k, float u) {
  const float ku = (float)(k + 2) * u;
  return ku / (1.f - ku) * (1.f + 4.f * u);
}

// butterfly sum within aligned groups of G lanes (every lane of the group gets the total)
template <int G>
__device__ __forceinline__ float fa_group_sum(float v) {
#pragma unroll
  for (int off = G / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// G lanes per box-row (G >= widest layer, up to 64): tiny networks (AC-8's 5-wide layers) pack
// 64 / G rows into one wave instead of leaving 59 of 64 lanes idle.  WP = per-row slab stride.
template <int G>
__global__ void __launch_bounds__(64 * FA_CROWN_WAVES) fa_crown_kernel(NetDesc net, BoundArgs a, int nparams, int WP) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int RPW = 64 / G;                                 // rows per wave
  const int tid = threadIdx.x;
  // stage W_l TRANSPOSED ([n_out][n_in]) so the lambda' = W mu loop (lanes over inputs i, loop
  // over outputs j) reads consecutive LDS words across lanes: the row-major copy made lanes
  // stride by n_out words (8-way bank conflicts for 100-wide layers, ~1/3 of the kernel's cycles
  // waiting on LDS, profiles/pmc/)
  for (int l = 0; l < net.n_layers; ++l) {
    const int nin = net.dims[l], nout = net.dims[l + 1];
    const float* src = a.flat + net.w_off[l];
    float* dst = smem + net.w_off[l];
    for (int e = tid; e < nin * nout; e += 64 * FA_CROWN_WAVES) {
      const int j = e / nin, i = e - j * nin;
      dst[e] = src[(size_t)i * nout + j];
    }
    for (int e = tid; e < nout; e += 64 * FA_CROWN_WAVES) smem[net.b_off[l] + e] = a.flat[net.b_off[l] + e];
  }
  __syncthreads();
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int grp = lane / G;
  const int gl = lane % G;
  // per-row slabs at an odd stride: groups of one wave reading lam/mu[j] at the same j hit
  // different banks
  float* lam = smem + nparams + (wave * RPW + grp) * (4 * WP + 1);   // [2][WP]
  float* mu = lam + 2 * WP;                                    // [2][WP]
  const int L = net.n_layers;
  const int n0 = net.dims[0];
  const int N = net.n_neurons;
  const float u = net.unit;
  const int rows_per_block = FA_CROWN_WAVES * RPW;
  for (int rb = blockIdx.x * rows_per_block; rb < a.R; rb += gridDim.x * rows_per_block) {
    const int r0 = rb + wave * RPW + grp;
    const bool valid = r0 < a.R;
    const int r = valid ? r0 : a.R - 1;            // idle groups shadow the last row, never write
    const int node = a.V > 0 ? r / a.V : r;
    const int v = a.V > 0 ? r - node * a.V : 0;
    const uint8_t* dmask = nullptr;                // forced-dead hidden neurons of this row
    if (a.dead_in) dmask = a.dead_in + (size_t)r * net.n_hidden;
    else if (a.dead_part) dmask = a.dead_part + (size_t)a.node_part[node] * net.n_hidden;
    const float* lbr = a.layer_lb + (size_t)r * N;
    const float* ubr = a.layer_ub + (size_t)r * N;
    // ---- init: lambda = +-W_{L-1}[:, 0], c = +-b_{L-1}
    {
      const int n = net.dims[L - 1];
      const float* W = smem + net.w_off[L - 1];
      for (int i = gl; i < n; i += G) {
        lam[i] = W[i];
        lam[WP + i] = -W[i];
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
      for (int j = gl; j < n; j += G) {
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
          const float lm = lam[sg * WP + j];
          const float slope = act ? 1.f : (dd ? 0.f : (lm >= 0.f ? alpha : s));
          const float m = lm * slope;
          const bool neg = unst && lm < 0.f;
          const float t = neg ? -m * lb : 0.f;
          mu[sg * WP + j] = m;
          cs[sg] += m * bj + t;
          cm[sg] += fabsf(m * bj) + fabsf(t);
          if (neg) er[sg] += 3.f * u * (fabsf(m) * zmax + fabsf(t));
        }
      }
      __builtin_amdgcn_wave_barrier();
      const float gn = fa_gam(n + 1, u);
      for (int i = gl; i < nin; i += G) {
        float acc0 = 0.f, acc1 = 0.f, mag0 = 0.f, mag1 = 0.f;
        for (int j = 0; j < n; ++j) {
          const float w = W[(size_t)j * nin + i];   // W^T in LDS
          const float m0 = mu[j], m1 = mu[WP + j];
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
        lam[WP + i] = acc1;
        er[0] += gn * mag0 * hm;
        er[1] += gn * mag1 * hm;
      }
      const float gc = fa_gam(2 * n + 1, u);
#pragma unroll
      for (int sg = 0; sg < 2; ++sg) {
        const float csum = fa_group_sum<G>(cs[sg]);
        const float cmag = fa_group_sum<G>(cm[sg]);
        const float esum = fa_group_sum<G>(er[sg]);
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
      for (int i = gl; i < n0; i += G) {
        float xl = a.lo[(size_t)node * n0 + i], xh = a.hi[(size_t)node * n0 + i];
        if (a.V > 0)
          for (int k = 0; k < a.npa; ++k)
            if (a.pa_idx[k] == i) xl = xh = a.values[v * a.npa + k];
        const float lm = lam[sg * WP + i];
        cp += fminf(lm * xl, lm * xh);
        mp += fabsf(lm) * fmaxf(fabsf(xl), fabsf(xh));
      }
      const float conc = fa_group_sum<G>(cp) + c[sg];
      const float cmg = fa_group_sum<G>(mp) + fabsf(c[sg]);
      err[sg] *= 1.f + 2.f * gK;
      low[sg] = conc - err[sg] - g0 * cmg - g1 * fabsf(conc);
    }
    if (valid) {
      const float olb = a.out_lb[r], oub = a.out_ub[r];
      const bool useL = low[0] >= olb;
      const bool useU = -low[1] <= oub;
      for (int i = gl; i < n0; i += G) {
        if (useL) a.Lc[(size_t)r * n0 + i] = lam[i];
        if (useU) a.Uc[(size_t)r * n0 + i] = -lam[WP + i];
      }
      if (gl == 0) {
        if (useL) { a.L0[r] = c[0]; a.Le[r] = err[0]; a.out_lb[r] = low[0]; }
        if (useU) { a.U0[r] = -c[1]; a.Ue[r] = err[1]; a.out_ub[r] = -low[1]; }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------------------------------------------------------------------
// MFMA variant: the back-substitution lambda' = W mu of 16 box-rows at once as GEMMs on
// v_mfma_f32_16x16x4_f32.  Rows are the 16 MFMA columns; a multiplier vector lives transposed in
// registers (reg i of tile t = neuron 16t + 4*(lane>>4) + i of row lane&15), so mu is formed
// elementwise in registers, W is the A operand (staged once per workgroup in LDS in operand order
// [ot][t][lane][i] = W[16ot + (lane&15)][16t + 4(lane>>4) + i]) and the accumulator tile of
// layer l IS the lambda of layer l-1 -- no LDS round trip for the vectors and no per-row
// serial dot products.  Two MFMA chains per sign: W mu and |W| |mu| (the rounding term).  Same
// relaxation choices and error terms as fa_crown_kernel, with the GEMM error bound taken for
// 2n+1 terms (the convention of the MFMA symbolic kernel).
struct CrownCfg {
  int w_lds[FA_MAX_LAYERS];   // LDS float offset of layer l's operand-order W (backward orientation)
  int b_lds[FA_MAX_LAYERS];
  int floats;
};

// Minimum waves per SIMD for the 4- and 7-tile kernels (VGPR budget 512 / waves): 220 -> 168
// and 338 -> 256 VGPRs with 80 / 160 B of scratch spills, 3 and 2 waves per SIMD instead of 2
// and 1: AC-4 0.71 -> 0.59 ms, AC-7 0.335 -> 0.31 ms per 131 072 rows (tools/ab_variants.sh,
// profiles/r2/occupancy.md).  -DFA_CROWN_WPE4=1 -DFA_CROWN_WPE7=1 restores the unconstrained build.
#ifndef FA_CROWN_WPE4
#define FA_CROWN_WPE4 3
#endif
#ifndef FA_CROWN_WPE7
#define FA_CROWN_WPE7 2
#endif
template <int TM>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(TM == 4 ? FA_CROWN_WPE4 : (TM == 7 ? FA_CROWN_WPE7 : 1)))) fa_crown_mfma_kernel(NetDesc net, BoundArgs a, CrownCfg cfg) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  // ---- stage every layer's W in backward operand order + biases
  for (int l = 0; l < net.n_layers; ++l) {
    const int nin = net.dims[l], nout = net.dims[l + 1];
    const int tin = (nin + 15) >> 4, tout = (nout + 15) >> 4;
    const float* W = a.flat + net.w_off[l];
    float* dst = smem + cfg.w_lds[l];
    const int tot = tin * tout * 256;
    for (int e = tid; e < tot; e += 256) {
      const int i4 = e & 3, ln = (e >> 2) & 63, tt = e >> 8;
      const int t = tt % tout, ot = tt / tout;
      const int in = 16 * ot + (ln & 15), out = 16 * t + 4 * (ln >> 4) + i4;
      dst[e] = (in < nin && out < nout) ? W[(size_t)in * nout + out] : 0.f;
    }
    for (int e = tid; e < nout; e += 256) smem[cfg.b_lds[l] + e] = a.flat[net.b_off[l] + e];
  }
  __syncthreads();
  const int lane = tid & 63, col = lane & 15, grp = lane >> 4;
  const int wave = tid >> 6;
  const int L = net.n_layers;
  const int n0 = net.dims[0];
  const int N = net.n_neurons;
  const float u = net.unit;
  const int ntile = (a.R + 15) >> 4;
  for (int tile = blockIdx.x * 4 + wave; tile < ntile; tile += gridDim.x * 4) {
    const int r0 = tile * 16 + col;
    const bool valid = r0 < a.R;
    const int r = valid ? r0 : a.R - 1;
    const int node = a.V > 0 ? r / a.V : r;
    const int v = a.V > 0 ? r - node * a.V : 0;
    if (a.skip_status) {   // BaB: skip tiles whose rows all belong to decided / stopped partitions
      const int8_t st = a.skip_status[a.skip_part[node]];
      if (!__any(valid && (st == 3 || st == 4))) continue;   // wave-uniform
    }
    const uint8_t* dmask = nullptr;
    if (a.dead_in) dmask = a.dead_in + (size_t)r * net.n_hidden;
    else if (a.dead_part) dmask = a.dead_part + (size_t)a.node_part[a.part_mod ? node % a.part_mod : node] * net.n_hidden;
    const float* lbr = a.layer_lb + (size_t)r * N;
    const float* ubr = a.layer_ub + (size_t)r * N;
    float lam[2][TM][4];
    // ---- init: lambda = +-W_{L-1}[:, 0], c = +-b_{L-1}
    {
      const int n = net.dims[L - 1];
      const float* W = a.flat + net.w_off[L - 1];
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int j = 16 * t + 4 * grp + i;
          const float w = j < n ? W[j] : 0.f;
          lam[0][t][i] = w;
          lam[1][t][i] = -w;
        }
    }
    float c[2], err[2];
    c[0] = smem[cfg.b_lds[L - 1]];
    c[1] = -c[0];
    err[0] = err[1] = 0.f;
    for (int l = L - 2; l >= 0; --l) {
      const int n = net.dims[l + 1];
      const int nin = net.dims[l];
      const int tout = (n + 15) >> 4, tin = (nin + 15) >> 4;
      const int off = net.neuron_off[l];
      const float* b = smem + cfg.b_lds[l];
      float mu[2][TM][4];
      float cs[2] = {0.f, 0.f}, cm[2] = {0.f, 0.f}, er[2] = {0.f, 0.f};
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int j = 16 * t + 4 * grp + i;
          const bool jv = t < tout && j < n;
          const float lb = jv ? lbr[off + j] : 0.f, ub = jv ? ubr[off + j] : 0.f;
          const bool dd = !jv || ub <= 0.f || (dmask && dmask[off + j]);
          const bool act = !dd && lb >= 0.f;
          const bool unst = !dd && !act;
          const float alpha = ub > -lb ? 1.f : 0.f;
          const float sl = unst ? (ub / (ub - lb)) * (1.f + 4.f * u) : 0.f;
          const float zmax = fmaxf(fabsf(lb), fabsf(ub));
          const float bj = jv ? b[j] : 0.f;
#pragma unroll
          for (int sg = 0; sg < 2; ++sg) {
            const float lm = lam[sg][t][i];
            const float slope = act ? 1.f : (dd ? 0.f : (lm >= 0.f ? alpha : sl));
            const float m = lm * slope;
            const bool neg = unst && lm < 0.f;
            const float tt = neg ? -m * lb : 0.f;
            mu[sg][t][i] = m;
            cs[sg] += m * bj + tt;
            cm[sg] += fabsf(m * bj) + fabsf(tt);
            if (neg) er[sg] += 3.f * u * (fabsf(m) * zmax + fabsf(tt));
          }
        }
      // lambda' = W mu and |W| |mu| (rounding term), both signs; |mu| once per layer
      float amu[2][TM][4];
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          amu[0][t][i] = fabsf(mu[0][t][i]);
          amu[1][t][i] = fabsf(mu[1][t][i]);
        }
      const float4* wb = reinterpret_cast<const float4*>(smem + cfg.w_lds[l]);
      const float gn = fa_gam(2 * n + 1, u);
#pragma unroll
      for (int ot = 0; ot < TM; ++ot) {
        if (ot >= tin) break;
        f32x4 Z0 = {0.f, 0.f, 0.f, 0.f}, Z1 = Z0, Q0 = Z0, Q1 = Z0;
#pragma unroll
        for (int t = 0; t < TM; ++t) {
          if (t >= tout) break;
          const float4 w4 = wb[(ot * tout + t) * 64 + lane];
          const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float aw = fabsf(wv[i]);
            Z0 = fa_mfma4(wv[i], mu[0][t][i], Z0);
            Z1 = fa_mfma4(wv[i], mu[1][t][i], Z1);
            Q0 = fa_mfma4(aw, amu[0][t][i], Q0);
            Q1 = fa_mfma4(aw, amu[1][t][i], Q1);
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int in = 16 * ot + 4 * grp + i;
          float hm = 0.f;
          if (in < nin) {
            if (l > 0) {
              const int po = net.neuron_off[l - 1];
              hm = fmaxf(ubr[po + in], 0.f);
              if (dmask && dmask[po + in]) hm = 0.f;
            } else {
              float xl = a.lo[(size_t)node * n0 + in], xh = a.hi[(size_t)node * n0 + in];
              if (a.V > 0)
                for (int k = 0; k < a.npa; ++k)
                  if (a.pa_idx[k] == in) xl = xh = a.values[v * a.npa + k];
              hm = fmaxf(fabsf(xl), fabsf(xh));
            }
          }
          lam[0][ot][i] = in < nin ? Z0[i] : 0.f;
          lam[1][ot][i] = in < nin ? Z1[i] : 0.f;
          er[0] += gn * Q0[i] * hm;
          er[1] += gn * Q1[i] * hm;
        }
      }
#pragma unroll
      for (int ot = 0; ot < TM; ++ot)       // tiles beyond the layer's inputs: zero
        if (ot >= tin)
#pragma unroll
          for (int i = 0; i < 4; ++i) lam[0][ot][i] = lam[1][ot][i] = 0.f;
      const float gc = fa_gam(2 * n + 1, u);
#pragma unroll
      for (int sg = 0; sg < 2; ++sg) {
        // per-row sums over the 4 lane groups holding this row's neurons
        float csum = cs[sg], cmag = cm[sg], esum = er[sg];
        csum += __shfl_xor(csum, 16); csum += __shfl_xor(csum, 32);
        cmag += __shfl_xor(cmag, 16); cmag += __shfl_xor(cmag, 32);
        esum += __shfl_xor(esum, 16); esum += __shfl_xor(esum, 32);
        const float cold = c[sg];
        c[sg] = cold + csum;
        err[sg] += esum + gc * (fabsf(cold) + cmag);
      }
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
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int in = 16 * t + 4 * grp + i;
          if (in >= n0) continue;
          float xl = a.lo[(size_t)node * n0 + in], xh = a.hi[(size_t)node * n0 + in];
          if (a.V > 0)
            for (int k = 0; k < a.npa; ++k)
              if (a.pa_idx[k] == in) xl = xh = a.values[v * a.npa + k];
          const float lm = lam[sg][t][i];
          cp += fminf(lm * xl, lm * xh);
          mp += fabsf(lm) * fmaxf(fabsf(xl), fabsf(xh));
        }
      cp += __shfl_xor(cp, 16); cp += __shfl_xor(cp, 32);
      mp += __shfl_xor(mp, 16); mp += __shfl_xor(mp, 32);
      const float conc = cp + c[sg];
      const float cmg = mp + fabsf(c[sg]);
      err[sg] *= 1.f + 2.f * gK;
      low[sg] = conc - err[sg] - g0 * cmg - g1 * fabsf(conc);
    }
    if (valid) {
      const float olb = a.out_lb[r], oub = a.out_ub[r];
      const bool useL = low[0] >= olb;
      const bool useU = -low[1] <= oub;
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int in = 16 * t + 4 * grp + i;
          if (in >= n0) continue;
          if (useL) a.Lc[(size_t)r * n0 + in] = lam[0][t][i];
          if (useU) a.Uc[(size_t)r * n0 + in] = -lam[1][t][i];
        }
      if (grp == 0) {
        if (useL) { a.L0[r] = c[0]; a.Le[r] = err[0]; a.out_lb[r] = low[0]; }
        if (useU) { a.U0[r] = -c[1]; a.Ue[r] = err[1]; a.out_ub[r] = -low[1]; }
      }
    }
  }
}

namespace {
typedef void (*CrownMfmaKernel)(NetDesc, BoundArgs, CrownCfg);
CrownMfmaKernel select_crown_mfma(int TM) {
  if (TM <= 1) return fa_crown_mfma_kernel<1>;
  if (TM <= 2) return fa_crown_mfma_kernel<2>;
  if (TM <= 4) return fa_crown_mfma_kernel<4>;
  if (TM <= 7) return fa_crown_mfma_kernel<7>;
  return nullptr;
}

int crown_cus() {
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

// 1 launched, 0 shape not supported by the MFMA variant, < 0 error
int crown_mfma_try(const NetDesc& net, const BoundArgs& a, hipStream_t stream) {
  static const bool off = [] {
    const char* e = getenv("FAIRIFY_CROWN_MFMA");
    return e && e[0] == '0';
  }();
  if (off) return 0;
  int TM = 1;
  for (int l = 0; l <= net.n_layers; ++l) TM = std::max(TM, (net.dims[l] + 15) / 16);
  CrownMfmaKernel k = select_crown_mfma(TM);
  if (!k) return 0;
  CrownCfg cfg{};
  int offs = 0;
  for (int l = 0; l < net.n_layers; ++l) {
    cfg.w_lds[l] = offs;
    offs += ((net.dims[l] + 15) / 16) * ((net.dims[l + 1] + 15) / 16) * 256;
  }
  for (int l = 0; l < net.n_layers; ++l) {
    cfg.b_lds[l] = offs;
    offs += net.dims[l + 1];
  }
  cfg.floats = (offs + 3) & ~3;
  const size_t bytes = (size_t)cfg.floats * sizeof(float);
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
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256, bytes) != hipSuccess || per_cu <= 0) per_cu = 1;
      occ[key] = per_cu;
    } else {
      per_cu = it->second;
    }
  }
  const long long tiles = (a.R + 15) / 16;
  long long blocks = (tiles + 3) / 4;
  const long long cap = (long long)crown_cus() * per_cu;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(256), bytes, stream, net, a, cfg);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 1 : -(int)e;
}
}  // namespace

// 0 on success; -1 if the network does not fit (a layer wider than FA_CROWN_MAXW or weights
// beyond the LDS budget) -- callers then keep the forward forms.
extern "C" int fa_crown_launch(const NetDesc& net, BoundArgs a, hipStream_t stream) {
  if (a.R <= 0) return 0;
  if (!a.layer_lb || !a.layer_ub || !a.Lc || !a.Uc) return -2;
  {
    const int rc = crown_mfma_try(net, a, stream);
    if (rc == 1) return 0;
    if (rc < 0) return -3;
  }
  int wmax = 1;
  for (int l = 0; l <= net.n_layers; ++l) {
    if (net.dims[l] > FA_CROWN_MAXW) return -1;
    if (l > 0) wmax = std::max(wmax, net.dims[l]);
  }
  // group size: smallest power of two >= the widest hidden/output layer (>= 4, <= 64)
  int G = 4;
  while (G < wmax && G < 64) G *= 2;
  const int WP = (std::max(wmax, net.dims[0]) + 3) & ~3;
  int nparams = 0;
  for (int l = 0; l < net.n_layers; ++l) nparams = net.b_off[l] + net.dims[l + 1];
  const int rows_per_block = FA_CROWN_WAVES * (64 / G);
  const size_t bytes = ((size_t)nparams + (size_t)rows_per_block * (4 * WP + 1)) * sizeof(float);
  if (bytes > 160 * 1024) return -1;
  typedef void (*K)(NetDesc, BoundArgs, int, int);
  K k = G == 4 ? fa_crown_kernel<4> : G == 8 ? fa_crown_kernel<8> : G == 16 ? fa_crown_kernel<16>
      : G == 32 ? fa_crown_kernel<32> : fa_crown_kernel<64>;
  if (!fa_lds_ok(bytes)) return -3;
  const int blocks = (int)std::min<long long>(((long long)a.R + rows_per_block - 1) / rows_per_block, 256LL * 8);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(64 * FA_CROWN_WAVES), bytes, stream, net, a, nparams, WP);
  return (int)hipGetLastError();
}

FA_LDS_REGISTER(FA_LDS_K(fa_crown_mfma_kernel<1>), FA_LDS_K(fa_crown_mfma_kernel<2>), FA_LDS_K(fa_crown_mfma_kernel<4>),
                FA_LDS_K(fa_crown_mfma_kernel<7>), FA_LDS_K(fa_crown_kernel<4>), FA_LDS_K(fa_crown_kernel<8>),
                FA_LDS_K(fa_crown_kernel<16>), FA_LDS_K(fa_crown_kernel<32>), FA_LDS_K(fa_crown_kernel<64>));
