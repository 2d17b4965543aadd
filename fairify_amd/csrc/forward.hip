// Concrete MLP forward on f32 MFMA + the fused simulation/falsification kernel.  gfx950.
//
// fa_forward_kernel : logits of arbitrary rows (candidate replay, accuracy, hybrid routing,
//                     causal testing; K7), with optional per-row dead-neuron masks
//                     (heuristically pruned networks).
// fa_sim_kernel     : one workgroup per partition; draws `S` lattice points with the counter
//                     RNG (never written to HBM), counts per-neuron activations (reference
//                     `candidate_dead_nodes`, utils/prune.py:168-192), re-evaluates each point
//                     under every protected-attribute value (+ relaxed offsets) and records the
//                     first strict sign flip (K3 + K8 fused).
// fa_ascent_kernel  : the residual falsifier's lattice coordinate ascent; one workgroup per
//                     partition keeps its K start points in LDS and runs every iteration
//                     (K x moves x PA values candidate rows through the MFMA tile forward,
//                     pair margins, best improving move per start) without leaving the kernel:
//                     one launch instead of ~10 launches and 2 host syncs per iteration.
//
// A 64-row tile goes through all layers in LDS; each layer is a 64 x n_in x n_out GEMM on
// v_mfma_f32_16x16x4_f32 with bias / ReLU / mask / activation counting fused into the
// accumulator epilogue (counts reduced across the 4 row-groups of a wave with shuffles, one LDS
// atomic per column per tile).
#include "args.h"
#include "regfwd.h"

#include <stdlib.h>

#define FA_TR 64

// rows [FA_TR][S] in bufA (cols 0..n0-1) -> logits in zout[FA_TR]; bufA/bufB clobbered.
// counts (optional): per-neuron activation counts over the valid rows, restricted to the rows
// with count_rows[r] != 0 when count_rows is given.
__device__ void fa_tile_forward(const NetDesc& net, const float* __restrict__ flat, float* bufA, float* bufB,
                                int S, int nvalid, const uint8_t* __restrict__ dead_rows, int dead_stride,
                                int* counts, float* zout, const uint8_t* count_rows = nullptr) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  for (int l = 0; l < net.n_layers; ++l) {
    const int n_in = net.dims[l];
    const int n_out = net.dims[l + 1];
    const float* __restrict__ W = flat + net.w_off[l];
    const float* __restrict__ bias = flat + net.b_off[l];
    const bool last = (l == net.n_layers - 1);
    const int noff = net.neuron_off[l];
    const int ntiles = (n_out + 15) >> 4;
    for (int t = wave; t < 4 * ntiles; t += 4) {
      const int mt = t / ntiles, nt = t % ntiles;
      const int m = mt * 16 + (lane & 15);
      const int kq = lane >> 4;
      const int j = nt * 16 + (lane & 15);
      const bool jval = j < n_out;
      const float* arow = bufA + m * S + kq;
      // columns j >= n_out read a valid column instead of a select per step (their accumulators
      // are never stored); full 4-wide K steps need no k < n_in test (same MFMA order and operands
      // as the predicated loop: bitwise the same logits and counts), only the tail keeps it
      const float* wcol = W + (size_t)kq * n_out + (jval ? j : n_out - 1);
      const int kfull = n_in & ~3;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int k0 = 0; k0 < kfull; k0 += 4)
        acc = fa_mfma4(arow[k0], wcol[(size_t)k0 * n_out], acc);
      if (kfull < n_in) {
        const bool kv = kfull + kq < n_in;
        const float av = kv ? arow[kfull] : 0.f;
        const float wv = kv ? wcol[(size_t)kfull * n_out] : 0.f;
        acc = fa_mfma4(av, wv, acc);
      }
      const float b = jval ? bias[j] : 0.f;
      int cnt = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = mt * 16 + (lane >> 4) * 4 + i;
        float v = acc[i] + b;
        if (!last) {
          v = fmaxf(v, 0.f);
          if (dead_rows && jval && r < nvalid && dead_rows[(size_t)r * dead_stride + noff + j]) v = 0.f;
        }
        if (jval) {
          if (last) zout[r] = v;
          else bufB[r * S + j] = v;
          cnt += (r < nvalid && v != 0.f && (!count_rows || count_rows[r])) ? 1 : 0;
        }
      }
      if (counts) {
        cnt += __shfl_xor(cnt, 16);
        cnt += __shfl_xor(cnt, 32);
        if (lane < 16 && jval) atomicAdd(&counts[noff + j], cnt);
      }
    }
    __syncthreads();
    float* tmp = bufA; bufA = bufB; bufB = tmp;
  }
}



__global__ void __launch_bounds__(FA_THREADS) fa_forward_kernel(NetDesc net, FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int S = a.S;
  float* bufA = smem;
  float* bufB = bufA + FA_TR * S;
  float* z = bufB + FA_TR * S;
  const int n0 = net.dims[0];
  const int r0 = blockIdx.x * FA_TR;
  const int nvalid = min(FA_TR, a.B - r0);
  for (int i = threadIdx.x; i < FA_TR * n0; i += FA_THREADS) {
    const int r = i / n0, d = i % n0;
    bufA[r * S + d] = (r < nvalid) ? a.x[(size_t)(r0 + r) * n0 + d] : 0.f;
  }
  __syncthreads();
  fa_tile_forward(net, a.flat, bufA, bufB, S, nvalid, a.dead ? a.dead + (size_t)r0 * net.n_hidden : nullptr,
                  net.n_hidden, nullptr, z);
  for (int i = threadIdx.x; i < nvalid; i += FA_THREADS) a.out[r0 + i] = z[i];
}

extern "C" int fa_forward_launch(const NetDesc& net, FwdArgs a, hipStream_t stream) {
  if (a.B <= 0) return 0;
  a.S = net.max_width | 1;
  size_t bytes = (2 * (size_t)FA_TR * a.S + FA_TR) * sizeof(float);
  if (!fa_lds_ok(bytes)) return -4;
  hipLaunchKernelGGL(fa_forward_kernel, dim3((a.B + FA_TR - 1) / FA_TR), dim3(FA_THREADS), bytes, stream, net, a);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------
#define FA_MAX_V 64



__device__ __forceinline__ float fa_sample_coord(uint32_t seed, int64_t pid, int s, int d, float lo, float hi) {
  const uint32_t h = fa_rng(seed, pid, s, d);
  const uint32_t w = (uint32_t)(hi - lo) + 1u;
  return lo + (float)(h % w);
}

// Witness of the first strict flip `key` = sample * Pp + pair of partition p (threads of one block).
__device__ void fa_sim_witness(const SimArgs& a, int n0, int p, int64_t pid, int key, const float* lo,
                               const float* hi) {
  const uint32_t seed_ra = a.seed ^ 0x2545F491u;
  const int s = key / a.Pp, q = key % a.Pp;
  const int vi = (int)a.pairs[2 * q], vj = (int)a.pairs[2 * q + 1];
  for (int d = threadIdx.x; d < n0; d += FA_THREADS) {
    const float base = fa_sample_coord(a.seed, pid, s, d, lo[d], hi[d]);
    float x = base, xp = base;
    for (int k = 0; k < a.npa; ++k)
      if (a.pa_idx[k] == d) {
        x = (float)a.values[vi * a.npa + k];
        xp = (float)a.values[vj * a.npa + k];
      }
    for (int k = 0; k < a.nra; ++k)
      if (a.ra_idx[k] == d) {
        const uint32_t h = fa_rng(seed_ra, pid, s, d);
        xp += (float)(h % (uint32_t)(2 * a.tau + 1)) - (float)a.tau;
      }
    a.wit_x[(size_t)p * n0 + d] = x;
    a.wit_xp[(size_t)p * n0 + d] = xp;
  }
}

// split > 1: `split` workgroups share one partition's sample tiles (tile t goes to group
// t % split), so a short residue list with a large sample budget still fills the 256 CUs.  The
// groups merge through global integer atomics (activation counts, min flip key), so the result
// is identical to split == 1; fa_sim_finalize_kernel then writes found / witness.
__global__ void __launch_bounds__(FA_THREADS) fa_sim_kernel(NetDesc net, SimArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int S = a.S;
  const int n0 = net.dims[0];
  const int G = a.split;
  const int p = blockIdx.x / G;
  const int g = blockIdx.x - p * G;
  const int tid = threadIdx.x;
  float* bufA = smem;
  float* bufB = bufA + FA_TR * S;
  float* X = bufB + FA_TR * S;              // [FA_TR][n0]
  float* z = X + FA_TR * n0;                // [FA_TR][V]
  float* zp = z + FA_TR * a.V;              // [FA_TR][V]
  float* zt = zp + FA_TR * a.V;             // [FA_TR]
  float* s_lo = zt + FA_TR;                 // [n0]
  float* s_hi = s_lo + n0;
  int* cnt = (int*)(s_hi + n0);             // [n_neurons]
  int* best = cnt + net.n_neurons;          // [1]
  uint8_t* cmatch = reinterpret_cast<uint8_t*>(best + 4);   // [FA_TR] sampled PA tuple == values[v]
  const int64_t pid = a.pids[p];
  for (int i = tid; i < n0; i += FA_THREADS) {
    s_lo[i] = a.lo[(size_t)p * n0 + i];
    s_hi[i] = a.hi[(size_t)p * n0 + i];
  }
  for (int i = tid; i < net.n_neurons; i += FA_THREADS) cnt[i] = 0;
  if (tid == 0) best[0] = 0x7FFFFFFF;
  __syncthreads();
  const uint32_t seed_ra = a.seed ^ 0x2545F491u;
  for (int s0 = g * FA_TR; s0 < a.n_samples; s0 += G * FA_TR) {
    const int nvalid = min(FA_TR, a.n_samples - s0);
    for (int i = tid; i < FA_TR * n0; i += FA_THREADS) {
      const int r = i / n0, d = i % n0;
      const float v = fa_sample_coord(a.seed, pid, s0 + r, d, s_lo[d], s_hi[d]);
      X[i] = v;
      bufA[r * S + d] = v;
    }
    __syncthreads();
    // falsification: every PA assignment (x) and, for relaxed queries, every x' variant.  The
    // profile (reference semantics: activation counts at the SAMPLED point) needs no pass of its
    // own: the values table holds every PA tuple of the box, so each sampled row equals exactly
    // one PA-assignment row of the first pass, whose activations are counted for it
    // (count_rows = cmatch) -- bitwise the same inputs, so the same counts with one forward pass
    // per tile fewer.
    const int passes = a.nra > 0 ? 2 : 1;
    for (int ps = 0; ps < passes; ++ps) {
      for (int v = 0; v < a.V; ++v) {
        for (int i = tid; i < FA_TR * n0; i += FA_THREADS) {
          const int r = i / n0, d = i % n0;
          float val = X[i];
          for (int k = 0; k < a.npa; ++k)
            if (a.pa_idx[k] == d) val = (float)a.values[v * a.npa + k];
          if (ps == 1) {
            for (int k = 0; k < a.nra; ++k)
              if (a.ra_idx[k] == d) {
                const uint32_t h = fa_rng(seed_ra, pid, s0 + r, d);
                val += (float)(h % (uint32_t)(2 * a.tau + 1)) - (float)a.tau;
              }
          }
          bufA[r * S + d] = val;
        }
        if (ps == 0)
          for (int r = tid; r < FA_TR; r += FA_THREADS) {
            bool m = true;
            for (int k = 0; k < a.npa; ++k) m = m && X[r * n0 + a.pa_idx[k]] == (float)a.values[v * a.npa + k];
            cmatch[r] = m ? 1 : 0;
          }
        __syncthreads();
        float* zdst = (ps == 0) ? z : zp;
        fa_tile_forward(net, a.flat, bufA, bufB, S, nvalid, nullptr, 0, ps == 0 ? cnt : nullptr, zt,
                        ps == 0 ? cmatch : nullptr);
        for (int r = tid; r < FA_TR; r += FA_THREADS) zdst[r * a.V + v] = zt[r];
        __syncthreads();
      }
    }
    const float* zq = (a.nra > 0) ? zp : z;
    if (a.z0)
      for (int r = tid; r < nvalid; r += FA_THREADS) a.z0[(size_t)p * a.n_samples + s0 + r] = z[r * a.V];
    for (int i = tid; i < nvalid * a.Pp; i += FA_THREADS) {
      const int r = i / a.Pp, q = i % a.Pp;
      const int vi = (int)a.pairs[2 * q], vj = (int)a.pairs[2 * q + 1];
      const float zi = z[r * a.V + vi], zj = zq[r * a.V + vj];
      if ((zi < 0.f && zj > 0.f) || (zi > 0.f && zj < 0.f)) atomicMin(best, (s0 + r) * a.Pp + q);
    }
    __syncthreads();
  }
  const int key = best[0];
  if (G > 1) {
    for (int i = tid; i < net.n_neurons; i += FA_THREADS)
      if (cnt[i]) atomicAdd(&a.counts[(size_t)p * net.n_neurons + i], cnt[i]);
    if (tid == 0 && key != 0x7FFFFFFF) atomicMin(&a.keys[p], key);
    return;
  }
  for (int i = tid; i < net.n_neurons; i += FA_THREADS) a.counts[(size_t)p * net.n_neurons + i] = cnt[i];
  if (tid == 0) a.found[p] = key != 0x7FFFFFFF;
  if (key != 0x7FFFFFFF) fa_sim_witness(a, n0, p, pid, key, s_lo, s_hi);
}

__global__ void __launch_bounds__(FA_THREADS) fa_sim_finalize_kernel(NetDesc net, SimArgs a) {
  const int n0 = net.dims[0];
  const int p = blockIdx.x;
  const int key = a.keys[p];
  if (threadIdx.x == 0) a.found[p] = key != 0x7FFFFFFF;
  if (key != 0x7FFFFFFF)
    fa_sim_witness(a, n0, p, a.pids[p], key, a.lo + (size_t)p * n0, a.hi + (size_t)p * n0);
}

// ------------------------------------------------------------------------------------------
// Register-resident simulation: the same samples (fa_sample_coord), PA passes,
// activation counts (at the sampled PA tuple) and first-flip keys as fa_sim_kernel, with 16
// samples per wave as the MFMA columns (csrc/regfwd.h): W staged once per workgroup in MFMA
// operand order, activations never leave registers, counts from one ballot per (tile, register)
// and layer (the 16 lanes of a lane group hold one neuron of the 16 samples).  The K grouping of
// the MFMA sums differs from the 64-row tile forward, so a logit within fp32 rounding of 0 may
// flip differently (counts stay within the rounding margins of tests/test_kernels_gpu.py).
// Relaxed queries add V passes of x' rows (fa_sim_kernel's offsets: x'_r = x_r + d, d uniform in
// [-tau, tau] from the seed ^ 0x2545F491 stream, unclipped), which are not counted.

// One layer with activation counting: H -> H2 (ReLU outputs); counts neuron j for the samples
// whose lanes have `match` (the sampled PA tuple is this pass's values[v]); last layer: the logit
// of sample lane&15 in lanes 0..15, counted when nonzero.
template <int TM>
__device__ __forceinline__ float fa_reg_layer_count(const NetDesc& net, const RegNetCfg& cfg, const float* sw_all,
                                                    int l, int lane, const float (&H)[TM][4], float (&H2)[TM][4],
                                                    bool match, int* cnt) {
  const int grp = lane >> 4, col = lane & 15;
  const int n_in = net.dims[l], n_out = net.dims[l + 1];
  const int tin = (n_in + 15) >> 4, tout = (n_out + 15) >> 4;
  const float4* sw = reinterpret_cast<const float4*>(sw_all + cfg.w_lds[l]);
  const float* sb = sw_all + cfg.b_lds[l];
  const bool last = l == net.n_layers - 1;
  const int noff = net.neuron_off[l];
  float logit = 0.f;
#pragma unroll
  for (int jt = 0; jt < TM; ++jt) {
    if (jt >= tout) break;
    f32x4 Z = {0.f, 0.f, 0.f, 0.f};
    const float4* wq = sw + (size_t)jt * tin * 64 + lane;
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      if (t >= tin) break;
      const float4 w4 = wq[t * 64];
      Z = fa_mfma4(w4.x, H[t][0], Z);
      Z = fa_mfma4(w4.y, H[t][1], Z);
      Z = fa_mfma4(w4.z, H[t][2], Z);
      Z = fa_mfma4(w4.w, H[t][3], Z);
    }
    if (last) {
      if (jt == 0) {
        logit = Z[0] + sb[0];
        const unsigned long long bm = __ballot(match && grp == 0 && logit != 0.f);
        if (lane == 0 && bm) atomicAdd(&cnt[noff], __popcll(bm));
      }
      continue;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = 16 * jt + 4 * grp + i;
      const float h = j >= n_out ? 0.f : fmaxf(Z[i] + sb[j], 0.f);
      H2[jt][i] = h;
      const unsigned long long bm = __ballot(match && h != 0.f);
      const int c = __popcll((bm >> (16 * grp)) & 0xFFFFull);
      if (col == 0 && c) atomicAdd(&cnt[noff + j], c);
    }
  }
  return logit;
}

template <int TM>
__global__ void __launch_bounds__(FA_THREADS) fa_sim_reg_kernel(NetDesc net, SimArgs a, RegNetCfg cfg) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, col = lane & 15, grp = lane >> 4;
  const int n0 = net.dims[0];
  const int G = a.split;
  const int p = blockIdx.x / G;
  const int g = blockIdx.x - p * G;
  const int V = a.V;
  const bool rx = a.nra > 0;
  const int RV = rx ? 2 * V : V;              // x rows, then (relaxed) x' rows per PA value
  const uint32_t seed_ra = a.seed ^ 0x2545F491u;
  const int64_t pid = a.pids[p];
  float* zs = smem + cfg.floats;              // [64][RV] logits of this pass's samples
  float* s_lo = zs + 64 * RV;
  float* s_hi = s_lo + n0;
  int* cnt = (int*)(s_hi + n0);               // [n_neurons]
  int* best = cnt + net.n_neurons;
  fa_stage_wperm(net, a.flat, smem, tid, FA_THREADS);
  for (int i = tid; i < n0; i += FA_THREADS) {
    s_lo[i] = a.lo[(size_t)p * n0 + i];
    s_hi[i] = a.hi[(size_t)p * n0 + i];
  }
  for (int i = tid; i < net.n_neurons; i += FA_THREADS) cnt[i] = 0;
  if (tid == 0) best[0] = 0x7FFFFFFF;
  __syncthreads();
  float Xb[TM][4], HA[TM][4], HB[TM][4];
  // which PA dim (if any) each of this lane's (tile, register) coordinates is, fixed for the launch
  // (hoisted out of the sample and pass loops: round 4 measured SALU:VALU 0.71 on this kernel)
  int8_t pslot[TM][4];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = 16 * t + 4 * grp + i;
      int q = -1;
      for (int m = 0; m < a.npa; ++m)
        if (a.pa_idx[m] == k) q = m;
      pslot[t][i] = (int8_t)q;
    }
  for (int s0 = g * FA_TR; s0 < a.n_samples; s0 += G * FA_TR) {
    const int s = s0 + wave * 16 + col;
    const bool sv = s < a.n_samples;
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = 16 * t + 4 * grp + i;
        Xb[t][i] = (k < n0 && sv) ? fa_sample_coord(a.seed, pid, s, k, s_lo[k], s_hi[k]) : 0.f;
      }
    // the pass whose PA tuple equals the sample's own: counted there (one hash per PA dim per
    // sample, not per pass)
    int vmatch = -1;
    if (sv) {
      float sp[FA_MAX_PA];
      for (int m = 0; m < a.npa; ++m) {
        const int d = a.pa_idx[m];
        sp[m] = fa_sample_coord(a.seed, pid, s, d, s_lo[d], s_hi[d]);
      }
      for (int v = 0; v < V && vmatch < 0; ++v) {
        bool eq = true;
        for (int m = 0; m < a.npa; ++m) eq = eq && sp[m] == (float)a.values[v * a.npa + m];
        if (eq) vmatch = v;
      }
    }
    for (int v2 = 0; v2 < RV; ++v2) {
      const int v = v2 < V ? v2 : v2 - V;
      const bool xp = v2 >= V;
      const bool match = !xp && v == vmatch;
      float vals[FA_MAX_PA];
      for (int m = 0; m < a.npa; ++m) vals[m] = (float)a.values[v * a.npa + m];
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = 16 * t + 4 * grp + i;
          float x = Xb[t][i];
          const int q = pslot[t][i];
          if (q >= 0) x = vals[q];
          if (xp && sv)
            for (int m = 0; m < a.nra; ++m)
              if (a.ra_idx[m] == k) x += (float)(fa_rng(seed_ra, pid, s, k) % (uint32_t)(2 * a.tau + 1)) - (float)a.tau;
          HA[t][i] = x;
        }
      float z = 0.f;
      for (int l = 0; l < net.n_layers; ++l) {
        if (l & 1) z = fa_reg_layer_count<TM>(net, cfg, smem, l, lane, HB, HA, match, cnt);
        else z = fa_reg_layer_count<TM>(net, cfg, smem, l, lane, HA, HB, match, cnt);
      }
      if (grp == 0) zs[(wave * 16 + col) * RV + v2] = z;   // read back by this same lane only
    }
    if (grp == 0 && sv) {
      const float* zr = zs + (wave * 16 + col) * RV;
      if (a.z0) a.z0[(size_t)p * a.n_samples + s] = zr[0];
      for (int q = 0; q < a.Pp; ++q) {
        const float zi = zr[(int)a.pairs[2 * q]], zj = zr[(rx ? V : 0) + (int)a.pairs[2 * q + 1]];
        if ((zi < 0.f && zj > 0.f) || (zi > 0.f && zj < 0.f)) {
          atomicMin(best, s * a.Pp + q);
          break;                                  // the sample's smallest flipping pair
        }
      }
    }
  }
  __syncthreads();
  const int key = best[0];
  if (G > 1) {
    for (int i = tid; i < net.n_neurons; i += FA_THREADS)
      if (cnt[i]) atomicAdd(&a.counts[(size_t)p * net.n_neurons + i], cnt[i]);
    if (tid == 0 && key != 0x7FFFFFFF) atomicMin(&a.keys[p], key);
    return;
  }
  for (int i = tid; i < net.n_neurons; i += FA_THREADS) a.counts[(size_t)p * net.n_neurons + i] = cnt[i];
  if (tid == 0) a.found[p] = key != 0x7FFFFFFF;
  if (key != 0x7FFFFFFF) fa_sim_witness(a, n0, p, pid, key, s_lo, s_hi);
}

namespace {
typedef void (*SimRegKernel)(NetDesc, SimArgs, RegNetCfg);
SimRegKernel select_sim_reg(int TM) {
  if (TM <= 1) return fa_sim_reg_kernel<1>;
  if (TM <= 2) return fa_sim_reg_kernel<2>;
  if (TM <= 4) return fa_sim_reg_kernel<4>;
  if (TM <= 7) return fa_sim_reg_kernel<7>;
  if (TM <= 10) return fa_sim_reg_kernel<10>;   // BM-4 (150-wide); the 64-row tile kernel before
  return nullptr;
}
// A/B switch (FAIRIFY_SIM_REG=0: the 64-row LDS tile kernel for every query)
bool sim_reg_on() {
  static const bool v = [] {
    const char* e = getenv("FAIRIFY_SIM_REG");
    return !(e && e[0] == '0');
  }();
  return v;
}
}  // namespace

extern "C" int fa_sim_launch(const NetDesc& net, SimArgs a, hipStream_t stream) {
  if (a.P <= 0) return 0;
  if (a.npa > FA_MAX_PA || a.nra > FA_MAX_RA) return -3;
  if ((long long)a.n_samples * a.Pp >= 0x7FFFFFFFLL) return -3;   // flip keys sample * Pp + pair are int
  a.S = net.max_width | 1;
  const int n0 = net.dims[0];
  if (sim_reg_on()) {
    const SimRegKernel k = select_sim_reg(fa_regnet_tm(net));
    RegNetCfg cfg{};
    if (k && fa_regnet_cfg(net, cfg)) {
      const size_t RV = a.nra > 0 ? 2 * (size_t)a.V : (size_t)a.V;
      size_t rb = ((size_t)cfg.floats + 64 * RV + 2 * n0) * sizeof(float) + (net.n_neurons + 4) * sizeof(int);
      rb = (rb + 15) & ~(size_t)15;
      const int tiles = (a.n_samples + FA_TR - 1) / FA_TR;
      if (rb <= 160 * 1024 && a.split >= 1 && (a.split == 1 || (a.keys && a.split <= tiles))) {
        if (!fa_lds_ok(rb)) return -4;
        hipLaunchKernelGGL(k, dim3((unsigned)a.P * (unsigned)a.split), dim3(FA_THREADS), rb, stream, net, a, cfg);
        if (a.split > 1) hipLaunchKernelGGL(fa_sim_finalize_kernel, dim3(a.P), dim3(FA_THREADS), 0, stream, net, a);
        return (int)hipGetLastError();
      }
    }
  }
  size_t floats = 2 * (size_t)FA_TR * a.S + (size_t)FA_TR * n0 + 2 * (size_t)FA_TR * a.V + FA_TR + 2 * n0;
  size_t bytes = floats * sizeof(float) + (net.n_neurons + 4) * sizeof(int) + FA_TR;
  bytes = (bytes + 15) & ~(size_t)15;
  if (bytes > 160 * 1024) return -1;
  if (!fa_lds_ok(bytes)) return -4;
  const int tiles = (a.n_samples + FA_TR - 1) / FA_TR;
  if (a.split < 1 || (a.split > 1 && (!a.keys || a.split > tiles))) return -2;
  hipLaunchKernelGGL(fa_sim_kernel, dim3((unsigned)a.P * (unsigned)a.split), dim3(FA_THREADS), bytes, stream, net, a);
  if (a.split > 1) hipLaunchKernelGGL(fa_sim_finalize_kernel, dim3(a.P), dim3(FA_THREADS), 0, stream, net, a);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// margin of a violation for ordered PA pair (vi, vj): min(-N(x, vi), N(x, vj)) > 0 iff strict flip
__global__ void __launch_bounds__(FA_THREADS) fa_ascent_kernel(NetDesc net, AscentArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int S = a.S;
  const int n0 = net.dims[0];
  const int K = a.K, V = a.V;
  const int nm = 2 * a.nfree;
  const int per = nm * V;                   // candidate rows per start
  const int total = K * per;
  const int p = blockIdx.x;
  const int tid = threadIdx.x;
  float* bufA = smem;
  float* bufB = bufA + FA_TR * S;
  float* zt = bufB + FA_TR * S;             // [FA_TR]
  float* X = zt + FA_TR;                    // [K][n0]
  float* F = X + K * n0;                    // [K]
  float* zall = F + K;                      // [K * nm * V]
  float* marg = zall + total;               // [K * nm]
  float* s_lo = marg + K * nm;              // [n0]
  float* s_hi = s_lo + n0;
  int* Q = (int*)(s_hi + n0);               // [K]
  int* margq = Q + K;                       // [K * nm]
  int* flag = margq + K * nm;               // [2]: any hit, any change
  for (int i = tid; i < n0; i += FA_THREADS) {
    s_lo[i] = a.lo[(size_t)p * n0 + i];
    s_hi[i] = a.hi[(size_t)p * n0 + i];
  }
  for (int i = tid; i < K * n0; i += FA_THREADS) X[i] = a.x0[(size_t)p * K * n0 + i];
  for (int i = tid; i < K; i += FA_THREADS) {
    F[i] = a.f0[(size_t)p * K + i];
    Q[i] = a.q0[(size_t)p * K + i];
  }
  __syncthreads();
  for (int it = 0; it < a.iters && nm > 0; ++it) {
    if (tid == 0) {
      int h = 0;
      for (int s = 0; s < K; ++s) h |= F[s] > 0.f;
      flag[0] = h;
      flag[1] = 0;
    }
    __syncthreads();
    if (flag[0]) break;                     // uniform: every thread reads the same LDS word
    for (int t0 = 0; t0 < total; t0 += FA_TR) {
      const int nvalid = min(FA_TR, total - t0);
      for (int i = tid; i < FA_TR * n0; i += FA_THREADS) {
        const int r = i / n0, d = i % n0;
        float val = 0.f;
        const int idx = t0 + r;
        if (r < nvalid) {
          const int v = idx % V;
          const int mv = (idx / V) % nm;
          const int s = idx / per;
          val = X[s * n0 + d];
          if (d == a.free_idx[mv >> 1]) val = fminf(fmaxf(val + ((mv & 1) ? 1.f : -1.f), s_lo[d]), s_hi[d]);
          for (int k = 0; k < a.npa; ++k)
            if (a.pa_idx[k] == d) val = (float)a.values[v * a.npa + k];
        }
        bufA[r * S + d] = val;
      }
      __syncthreads();
      fa_tile_forward(net, a.flat, bufA, bufB, S, nvalid, nullptr, 0, nullptr, zt);
      for (int r = tid; r < nvalid; r += FA_THREADS) zall[t0 + r] = zt[r];
      __syncthreads();
    }
    // best pair per (start, move); first index on ties
    for (int i = tid; i < K * nm; i += FA_THREADS) {
      const float* z = zall + (size_t)i * V;
      float g = -INFINITY;
      int gq = 0;
      for (int q = 0; q < a.Pp; ++q) {
        const float m = fminf(-z[a.pairs[2 * q]], z[a.pairs[2 * q + 1]]);
        if (m > g) { g = m; gq = q; }
      }
      marg[i] = g;
      margq[i] = gq;
    }
    __syncthreads();
    // best improving move per start
    for (int s = tid; s < K; s += FA_THREADS) {
      float g = -INFINITY;
      int gm = 0;
      for (int mv = 0; mv < nm; ++mv)
        if (marg[s * nm + mv] > g) { g = marg[s * nm + mv]; gm = mv; }
      if (g > F[s]) {
        const int d = a.free_idx[gm >> 1];
        X[s * n0 + d] = fminf(fmaxf(X[s * n0 + d] + ((gm & 1) ? 1.f : -1.f), s_lo[d]), s_hi[d]);
        F[s] = g;
        Q[s] = margq[s * nm + gm];
        flag[1] = 1;
      }
    }
    __syncthreads();
    if (!flag[1]) break;
    __syncthreads();
  }
  // witness: the first start with a strictly positive margin
  __syncthreads();
  int sh = -1;
  for (int s = 0; s < K; ++s)
    if (F[s] > 0.f) { sh = s; break; }
  if (tid == 0) a.found[p] = sh >= 0;
  if (sh >= 0) {
    const int q = Q[sh];
    const int vi = (int)a.pairs[2 * q], vj = (int)a.pairs[2 * q + 1];
    for (int d = tid; d < n0; d += FA_THREADS) {
      float x = X[sh * n0 + d], xp = x;
      for (int k = 0; k < a.npa; ++k)
        if (a.pa_idx[k] == d) {
          x = (float)a.values[vi * a.npa + k];
          xp = (float)a.values[vj * a.npa + k];
        }
      a.wit_x[(size_t)p * n0 + d] = x;
      a.wit_xp[(size_t)p * n0 + d] = xp;
    }
  }
}

// 0 on success, -1 if the candidate rows of one partition do not fit in LDS (callers keep the
// PyTorch path), -3 on bad arguments
extern "C" int fa_ascent_launch(const NetDesc& net, AscentArgs a, hipStream_t stream) {
  if (a.P <= 0) return 0;
  if (a.npa > FA_MAX_PA || a.nfree > 64 || a.K <= 0 || a.V <= 0 || a.Pp <= 0) return -3;
  a.S = net.max_width | 1;
  const int n0 = net.dims[0];
  const size_t nm = 2 * (size_t)a.nfree;
  const size_t floats = 2 * (size_t)FA_TR * a.S + FA_TR + (size_t)a.K * n0 + a.K + (size_t)a.K * nm * a.V +
                        (size_t)a.K * nm + 2 * (size_t)n0;
  size_t bytes = floats * sizeof(float) + ((size_t)a.K + (size_t)a.K * nm + 2) * sizeof(int);
  bytes = (bytes + 15) & ~(size_t)15;
  if (bytes > 160 * 1024) return -1;
  if (!fa_lds_ok(bytes)) return -4;
  hipLaunchKernelGGL(fa_ascent_kernel, dim3(a.P), dim3(FA_THREADS), bytes, stream, net, a);
  return (int)hipGetLastError();
}

FA_LDS_REGISTER(FA_LDS_K(fa_forward_kernel), FA_LDS_K(fa_sim_kernel), FA_LDS_K(fa_ascent_kernel),
                FA_LDS_K(fa_sim_reg_kernel<1>), FA_LDS_K(fa_sim_reg_kernel<2>), FA_LDS_K(fa_sim_reg_kernel<4>),
                FA_LDS_K(fa_sim_reg_kernel<7>), FA_LDS_K(fa_sim_reg_kernel<10>));
