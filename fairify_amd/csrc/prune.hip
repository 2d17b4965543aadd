// Pruning-stage kernels (K5 + the sound-prune mask algebra + the Pruned-acc replay).  gfx950.
//
// fa_prune_masks_kernel  one thread per partition: the sound-prune mask algebra of the pipeline's
//                        stage 2 in one pass (engine/prune.py: candidates_from_counts, bound_dead,
//                        ensure_one_alive, merge; reference utils/prune.py:168-251,671-859):
//                          cand    = never active in the simulation (counts == 0)
//                          b_dead  = cand & IBP ub <= 0 (hidden), cand (output), one alive per layer
//                          s_dead  = cand & !b & symbolic-dead (hidden)
//                          st_dead = b_dead | s_dead, one alive per layer;  s_cand = cand & !b & !s
//                        packed as bit codes per neuron plus the three dead counts per partition.
// fa_heuristic_kernel    one wave64 per UNKNOWN partition: the reference's heuristic pruning
//                        (utils/prune.py:862-939, engine/prune.py:heuristic_prune_batch) -- per hidden
//                        layer, means / NumPy-'linear' percentiles of the candidates' and the
//                        non-candidates' IBP upper bounds (fp64, ranks by counting in LDS), harsh
//                        outliers marked dead, merged with the sound masks, one alive per layer.
// fa_agree_kernel        one workgroup per partition: Pruned-acc = sign agreement of the full and
//                        the pruned network on the partition's simulation points (same
//                        counter-hash stream), plus the true / false positives of the pruned
//                        labels against the original's (Pruned F1 of the experiment drivers),
//                        register-resident MFMA forward (csrc/regfwd.h), dead mask in LDS.
#include <hip/hip_runtime.h>

#include "regfwd.h"

#define PM_CAND 1
#define PM_B 2
#define PM_S 4
#define PM_ST 8
#define PM_SCAND 16

// layer boundaries of the all-neuron numbering (hidden layers, then the output neuron)
__device__ __forceinline__ int fa_layer_end(const NetDesc& net, int l) { return net.neuron_off[l] + net.dims[l + 1]; }

__global__ void __launch_bounds__(FA_THREADS) fa_prune_masks_kernel(NetDesc net, int P, const int* counts,
                                                                   const float* ub, int ub_stride,
                                                                   const uint8_t* sym_dead, uint8_t* code,
                                                                   int* cnt) {
  const int p = blockIdx.x * FA_THREADS + threadIdx.x;
  if (p >= P) return;
  const int N = net.n_neurons, Nh = net.n_hidden;
  const int* c = counts + (size_t)p * N;
  const float* u = ub + (size_t)p * ub_stride;
  const uint8_t* sd = sym_dead ? sym_dead + (size_t)p * Nh : nullptr;
  uint8_t* out = code + (size_t)p * N;
  int nb = 0, ns = 0, nst = 0;
  for (int l = 0; l < net.n_layers; ++l) {
    const int j0 = net.neuron_off[l], j1 = fa_layer_end(net, l);
    const bool hidden = l < net.n_layers - 1;
    bool all_b = true, all_st = true;
    for (int j = j0; j < j1; ++j) {
      const bool cand = c[j] == 0;
      bool b, s;
      if (hidden) {
        b = cand && u[j] <= 0.f;
        s = cand && !b && sd && sd[j];
      } else {
        b = cand;           // output layer: the reference keeps the candidate flag (utils/prune.py:233-240)
        s = false;
      }
      uint8_t v = (cand ? PM_CAND : 0) | (b ? PM_B : 0) | (s ? PM_S : 0) | ((b || s) ? PM_ST : 0);
      if (cand && !b && !s) v |= PM_SCAND;
      if (!hidden && cand) v |= PM_SCAND;   // output neuron: s_cand keeps the bound stage's remainder
      out[j] = v;
      all_b = all_b && b;
      all_st = all_st && (b || s);
    }
    if (all_b) out[j0] &= (uint8_t)~PM_B;     // ensure_one_alive (utils/prune.py:689-691)
    if (all_st) out[j0] &= (uint8_t)~PM_ST;
    for (int j = j0; j < j1; ++j) {
      nb += (out[j] & PM_B) != 0;
      ns += (out[j] & PM_S) != 0;
      nst += (out[j] & PM_ST) != 0;
    }
  }
  cnt[3 * p + 0] = nb;
  cnt[3 * p + 1] = ns;
  cnt[3 * p + 2] = nst;
}

// ---------------------------------------------------------------------------------------------
#define FA_HEUR_MAXW 512

// value at sorted position `pos` (NumPy 'linear') of the k ranked entries in `srt`
__device__ __forceinline__ double fa_pct(const double* srt, int k, double q) {
  const int kk = k > 1 ? k : 1;
  const double pos = __dmul_rn((double)(kk - 1), q);
  const int lo = (int)floor(pos);
  const int hi = lo + 1 < kk - 1 ? lo + 1 : kk - 1;
  const double frac = __dsub_rn(pos, (double)lo);
  const double a = k > 0 ? srt[lo] : INFINITY, b = k > 0 ? srt[hi] : INFINITY;
  return __dadd_rn(a, __dmul_rn(__dsub_rn(b, a), frac));
}

__global__ void __launch_bounds__(64) fa_heuristic_kernel(NetDesc net, int Pu, const int64_t* rows, const float* lb,
                                                          const float* ub, int stride, const uint8_t* code,
                                                          double q50, double qlo, double qhi, uint8_t* hnew,
                                                          uint8_t* hmerged, int* hcnt) {
  __shared__ double su[FA_HEUR_MAXW], sl[FA_HEUR_MAXW], sc[FA_HEUR_MAXW], sn[FA_HEUR_MAXW];
  __shared__ uint8_t scode[FA_HEUR_MAXW], snew[FA_HEUR_MAXW];
  const int k = blockIdx.x;
  if (k >= Pu) return;
  const int lane = threadIdx.x;
  const int64_t p = rows[k];
  const int N = net.n_neurons;
  uint8_t* on = hnew + (size_t)k * N;
  uint8_t* om = hmerged + (size_t)k * N;
  int n_new = 0, n_merged = 0;
  for (int l = 0; l < net.n_layers; ++l) {
    const int j0 = net.neuron_off[l], w = net.dims[l + 1];
    const bool hidden = l < net.n_layers - 1;
    for (int i = lane; i < w; i += 64) {
      su[i] = (double)ub[(size_t)p * stride + j0 + i];
      sl[i] = (double)lb[(size_t)p * stride + j0 + i];
      scode[i] = code[(size_t)p * N + j0 + i];
      snew[i] = 0;
    }
    __syncthreads();
    if (hidden) {
      // candidate / non-candidate counts and sums (fp64)
      int kc = 0, kn = 0;
      double sum_c = 0.0, sum_n = 0.0;
      for (int i = 0; i < w; ++i) {   // every lane the same serial order: identical results
        if (scode[i] & PM_CAND) { ++kc; sum_c += su[i]; }
        else { ++kn; sum_n += su[i]; }
      }
      // ranks by counting (ties by index) -> sorted copies of both groups
      for (int i = lane; i < w; i += 64) {
        const bool ci = (scode[i] & PM_CAND) != 0;
        int r = 0;
        for (int t = 0; t < w; ++t) {
          if (((scode[t] & PM_CAND) != 0) != ci) continue;
          r += (su[t] < su[i]) || (su[t] == su[i] && t < i);
        }
        if (ci) sc[r] = su[i];
        else sn[r] = su[i];
      }
      __syncthreads();
      if (kn == 0) {
        for (int i = lane; i < w; i += 64) snew[i] = 1;
      } else if (kc > 0) {
        const double mean_c = sum_c / (double)kc, mean_n = sum_n / (double)kn;
        const double med_c = fa_pct(sc, kc, q50), med_n = fa_pct(sn, kn, q50);
        const double p5 = fa_pct(sn, kn, qlo), p95 = fa_pct(sn, kn, qhi);
        if (mean_n > 2.0 * mean_c && med_n > 2.0 * med_c)
          for (int i = lane; i < w; i += 64)
            snew[i] = (scode[i] & PM_SCAND) && su[i] < p5 && su[i] < 0.1 * p95 && su[i] < fabs(sl[i]);
      }
    }
    __syncthreads();
    // one alive per layer: new, then merged = sound (st) | new
    bool all_new = true, all_m = true;
    for (int i = 0; i < w; ++i) {
      all_new = all_new && snew[i];
      all_m = all_m && (snew[i] || (scode[i] & PM_ST));
    }
    for (int i = lane; i < w; i += 64) {
      const uint8_t nv = (snew[i] && !(all_new && i == 0)) ? 1 : 0;
      const uint8_t mv = ((nv || (scode[i] & PM_ST)) && !(all_m && i == 0)) ? 1 : 0;
      on[j0 + i] = nv;
      om[j0 + i] = mv;
    }
    for (int i = 0; i < w; ++i) {
      const bool nv = snew[i] && !(all_new && i == 0);
      n_new += nv;
      n_merged += (nv || (scode[i] & PM_ST)) && !(all_m && i == 0);
    }
    __syncthreads();
  }
  if (lane == 0) {
    hcnt[2 * k + 0] = n_new;
    hcnt[2 * k + 1] = n_merged;
  }
}

// ---------------------------------------------------------------------------------------------
template <int TM>
__global__ void __launch_bounds__(FA_THREADS) fa_agree_kernel(NetDesc net, RegNetCfg cfg, const float* flat, int Pm,
                                                              const int64_t* rows,
                                                              const float* lo, const float* hi, const int64_t* pids,
                                                              const uint8_t* dead, int S, uint32_t seed, int* agree) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, col = lane & 15, grp = lane >> 4;
  const int k = blockIdx.x;
  const int n0 = net.dims[0], Nh = net.n_hidden;
  const int64_t p = rows[k];
  const int64_t pid = pids[p];
  float* s_lo = smem + cfg.floats;
  float* s_hi = s_lo + n0;
  int* acc = (int*)(s_hi + n0);
  uint8_t* dm = (uint8_t*)(acc + 4);
  fa_stage_wperm(net, flat, smem, tid, FA_THREADS);
  for (int i = tid; i < n0; i += FA_THREADS) {
    s_lo[i] = lo[(size_t)p * n0 + i];
    s_hi[i] = hi[(size_t)p * n0 + i];
  }
  for (int i = tid; i < Nh; i += FA_THREADS) dm[i] = dead[(size_t)k * Nh + i];
  if (tid < 4) acc[tid] = 0;
  __syncthreads();
  int mine = 0, tp = 0, fp = 0;
  float HA[TM][4], HB[TM][4], X[TM][4];
  for (int s0 = wave * 16; s0 < S; s0 += 64) {
    const int s = s0 + col;
    const bool sv = s < S;
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int d = 16 * t + 4 * grp + i;
        float x = 0.f;
        if (d < n0 && sv) {
          const uint32_t h = fa_rng(seed, pid, s, d);
          x = s_lo[d] + (float)(h % ((uint32_t)(s_hi[d] - s_lo[d]) + 1u));
        }
        X[t][i] = x;
        HA[t][i] = x;
      }
    const float z0 = fa_reg_forward<TM>(net, cfg, smem, lane, HA, HB);
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) HA[t][i] = X[t][i];
    const float z1 = fa_reg_forward<TM>(net, cfg, smem, lane, HA, HB, dm);
    if (grp == 0 && sv) {
      mine += ((z0 > 0.f) == (z1 > 0.f)) ? 1 : 0;
      tp += (z0 > 0.f && z1 > 0.f) ? 1 : 0;       // F1 of the pruned labels against the original's
      fp += (z0 <= 0.f && z1 > 0.f) ? 1 : 0;
    }
  }
  atomicAdd(&acc[0], mine);
  atomicAdd(&acc[1], tp);
  atomicAdd(&acc[2], fp);
  __syncthreads();
  if (tid < 3) agree[3 * k + tid] = acc[tid];
}

namespace {
typedef void (*AgreeKernel)(NetDesc, RegNetCfg, const float*, int, const int64_t*, const float*, const float*, const int64_t*,
                            const uint8_t*, int, uint32_t, int*);
AgreeKernel select_agree(int TM) {
  if (TM <= 1) return fa_agree_kernel<1>;
  if (TM <= 2) return fa_agree_kernel<2>;
  if (TM <= 4) return fa_agree_kernel<4>;
  if (TM <= 7) return fa_agree_kernel<7>;
  return nullptr;
}
}  // namespace

extern "C" int fa_prune_masks_launch(const NetDesc& net, int P, const int* counts, const float* ub, int ub_stride,
                                     const uint8_t* sym_dead, uint8_t* code, int* cnt, hipStream_t stream) {
  if (P <= 0) return 0;
  if (ub_stride < net.n_hidden) return -3;
  hipLaunchKernelGGL(fa_prune_masks_kernel, dim3((P + FA_THREADS - 1) / FA_THREADS), dim3(FA_THREADS), 0, stream, net,
                     P, counts, ub, ub_stride, sym_dead, code, cnt);
  return (int)hipGetLastError();
}

extern "C" int fa_heuristic_launch(const NetDesc& net, int Pu, const int64_t* rows, const float* lb, const float* ub,
                                   int stride, const uint8_t* code, double q50, double qlo, double qhi, uint8_t* hnew,
                                   uint8_t* hmerged, int* hcnt, hipStream_t stream) {
  if (Pu <= 0) return 0;
  for (int l = 0; l < net.n_layers; ++l)
    if (net.dims[l + 1] > FA_HEUR_MAXW) return -4;
  if (stride < net.n_neurons) return -3;
  hipLaunchKernelGGL(fa_heuristic_kernel, dim3(Pu), dim3(64), 0, stream, net, Pu, rows, lb, ub, stride, code, q50, qlo,
                     qhi, hnew, hmerged, hcnt);
  return (int)hipGetLastError();
}

// 1 launched, 0 unsupported shape (caller keeps the PyTorch path), < 0 error
extern "C" int fa_agree_launch(const NetDesc& net, const float* flat, int Pm, const int64_t* rows, const float* lo, const float* hi,
                               const int64_t* pids, const uint8_t* dead, int S, uint32_t seed, int* agree,
                               hipStream_t stream) {
  if (Pm <= 0) return 1;
  AgreeKernel k = select_agree(fa_regnet_tm(net));
  if (!k) return 0;
  RegNetCfg cfg{};
  if (!fa_regnet_cfg(net, cfg)) return -1;
  const size_t bytes = ((size_t)cfg.floats + 2 * net.dims[0] + 4) * sizeof(float) + net.n_hidden + 16;
  if (bytes > 160 * 1024) return 0;
  if (!fa_lds_ok(bytes)) return -4;
  hipLaunchKernelGGL(k, dim3((unsigned)Pm), dim3(FA_THREADS), bytes, stream, net, cfg, flat, Pm, rows, lo, hi, pids, dead, S,
                     seed, agree);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 1 : -(int)e;
}

FA_LDS_REGISTER(FA_LDS_K(fa_agree_kernel<1>), FA_LDS_K(fa_agree_kernel<2>), FA_LDS_K(fa_agree_kernel<4>),
                FA_LDS_K(fa_agree_kernel<7>));
