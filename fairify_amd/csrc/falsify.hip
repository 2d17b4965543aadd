// Fused residual falsifier (K8): one kernel launch per residue list instead of a simulation
// kernel + ~1 000 PyTorch ops per work item (boundary walk and local-search set-up in
// engine/falsify.py, profiles/r2/ops_per_stage.md).  gfx950, non-relaxed queries.
//
// One workgroup (4 wave64) per partition; the network runs register-resident (csrc/regfwd.h):
// each wave pushes 16 lattice points at a time through the MFMA tiles with W staged once in LDS.
//
//   1  heavy sampling: n_samples counter-hash points (the simulation stream, engine/sim.py), every
//      PA assignment; the first strict flip (sample-major, then pair) is the witness.  Rounds of
//      64 samples stop as soon as a round produced a flip: later samples have larger keys, so the
//      witness equals the full pass's.  Keeps z0 (logit at PA value 0) and the best pair margin
//      min(-N(x, v), N(x, v')) of the first n_local samples.
//   2  boundary walk (no flip yet): bisection on the lattice between the walk_k samples of
//      largest and of smallest z0 (engine/sim.py:boundary_walk), every PA assignment per probe.
//   3  local search (still none): coordinate ascent from the K best-margin samples among the
//      first n_local, +-1 moves on every free dimension, all rounds inside the kernel
//      (engine/falsify.py:_local_search, same moves and acceptance rule as fa_ascent_kernel).
//
// Relaxed queries (|x_r - x'_r| <= tau on the RA dims, x' unclipped): every point carries its RA
// offsets d (sample: hash stream dseed, like engine/falsify.py; local search: +-1 moves clamped to
// [-tau, tau]); a point is evaluated as V rows of x and V rows of x', and a pair (v, v') counts in
// both orientations, N(x, v) < 0 < N(x', v') or N(x, v) > 0 > N(x', v').  The boundary walk probes
// x' = x (d = 0, always admissible).
//
// Only the witness is reported; the pipeline confirms it exactly (engine/exact.py).
#include <hip/hip_runtime.h>

#include <climits>

#include "regfwd.h"

namespace {

struct FalsifyLds {
  int z0, fm, fq, zs, slo, shi, wa, wb, tlo, thi, wok, widx, sval, X, F, Q, marg, margq, misc, DK, floats;
};

__host__ __device__ inline bool fa_fals_relaxed(const FalsifyArgs& a) { return a.nra > 0 && a.tau > 0; }

// Offsets (floats) of the kernel's LDS arrays after the staged weights; identical on host/device.
__host__ __device__ inline FalsifyLds fa_falsify_lds(const FalsifyArgs& a, int n0, int wfloats) {
  FalsifyLds L;
  const int nl = a.n_local < a.n_samples ? a.n_local : a.n_samples;
  const int kw = a.walk_k < a.n_samples ? a.walk_k : a.n_samples;
  const int K = a.K < nl ? a.K : nl;
  const bool rx = fa_fals_relaxed(a);
  const int nm = 2 * a.nfree + (rx ? 2 * a.nra : 0);
  const int RV = rx ? 2 * a.V : a.V;              // rows per point: x (and x') per PA value
  int o = wfloats;
  L.z0 = o; o += a.n_samples;
  L.fm = o; o += nl;
  L.fq = o; o += nl;
  const int zs1 = 4 * 16 * RV, zs2 = K * nm * RV, zs3 = kw * a.V;
  int zs = zs1 > zs2 ? zs1 : zs2;
  zs = zs > zs3 ? zs : zs3;
  L.zs = o; o += zs;
  L.slo = o; o += n0;
  L.shi = o; o += n0;
  L.wa = o; o += kw * n0;
  L.wb = o; o += kw * n0;
  L.tlo = o; o += kw;
  L.thi = o; o += kw;
  L.wok = o; o += kw;
  L.widx = o; o += (2 * kw > K ? 2 * kw : K);     // selected sample indices (walk, then starts)
  L.sval = o; o += (kw > K ? kw : K);             // their values while masked
  L.X = o; o += K * n0;
  L.F = o; o += K;
  L.Q = o; o += K;
  L.marg = o; o += K * nm;
  L.margq = o; o += K * nm;
  L.DK = o; o += rx ? K * a.nra : 0;
  L.misc = o; o += 8;
  L.floats = (o + 3) & ~3;
  return L;
}

__device__ __forceinline__ float fa_coord(uint32_t seed, int64_t pid, int s, int d, float lo, float hi) {
  const uint32_t h = fa_rng(seed, pid, s, d);
  return lo + (float)(h % ((uint32_t)(hi - lo) + 1u));
}

// PA dim d -> index into the PA list, or -1
__device__ __forceinline__ int fa_pa_slot(const FalsifyArgs& a, int d) {
  int r = -1;
  for (int m = 0; m < a.npa; ++m)
    if (a.pa_idx[m] == d) r = m;
  return r;
}

// RA dim d -> index into the RA list, or -1 (relaxed queries only)
__device__ __forceinline__ int fa_ra_slot(const FalsifyArgs& a, int d) {
  int r = -1;
  for (int m = 0; m < a.nra; ++m)
    if (a.ra_idx[m] == d) r = m;
  return r;
}

// sample s's offset on RA slot m: uniform in [-tau, tau] (engine/falsify.py: rng_u32(dseed, pid, s,
// ra_idx[m]) % (2 tau + 1) - tau)
__device__ __forceinline__ float fa_roff(const FalsifyArgs& a, int64_t pid, int s, int m) {
  return (float)(fa_rng(a.dseed, pid, s, a.ra_idx[m]) % (uint32_t)(2 * a.tau + 1)) - (float)a.tau;
}

// best margin over the pairs of one point from its row logits zr (x rows [0, V), x' rows [V, 2V)
// when relaxed): returns max over pairs (and orientations) of min(-N(x, v), N(x', v')) /
// min(N(x, v), -N(x', v')); *gq = the pair index, *flip = first strictly violating pair or -1
__device__ __forceinline__ float fa_pair_margin(const FalsifyArgs& a, const float* zr, bool rx, int* gq, int* flip) {
  float g = -INFINITY;
  int q0 = 0, fk = -1;
  for (int q = 0; q < a.Pp; ++q) {
    const float zi = zr[(int)a.pairs[2 * q]];
    const float zj = zr[(rx ? a.V : 0) + (int)a.pairs[2 * q + 1]];
    float mg = fminf(-zi, zj);
    if (rx) mg = fmaxf(mg, fminf(zi, -zj));
    if (mg > g) { g = mg; q0 = q; }
    if (fk < 0 && ((zi < 0.f && zj > 0.f) || (zi > 0.f && zj < 0.f))) fk = q;
  }
  *gq = q0;
  *flip = fk;
  return g;
}

// wave-wide (value, index) selection: the largest value (sign = +1) or the smallest (sign = -1),
// ties to the lower index; every lane returns the winner
__device__ __forceinline__ void fa_wave_pick(float& v, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float v2 = __shfl_xor(v, o);
    const int i2 = __shfl_xor(i, o);
    if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
  }
}

// Wave 0 selects the k extreme entries of buf[0..n) (sign +1: largest first, -1: smallest
// first) into out[0..k); entries are masked while selecting and restored afterwards.
__device__ void fa_select_extremes(float* buf, int n, int k, float sign, int* out, float* saved, int lane) {
  for (int j = 0; j < k; ++j) {
    float bv = -INFINITY;
    int bi = INT_MAX;
    for (int s = lane; s < n; s += 64) {
      const float v = sign * buf[s];
      if (v > bv || (v == bv && s < bi)) { bv = v; bi = s; }
    }
    fa_wave_pick(bv, bi);
    if (lane == 0) {
      out[j] = bi;
      saved[j] = buf[bi];
      buf[bi] = -sign * INFINITY;   // never selected again
    }
    __builtin_amdgcn_wave_barrier();
  }
  __builtin_amdgcn_wave_barrier();
  if (lane == 0)
    for (int j = k - 1; j >= 0; --j) buf[out[j]] = saved[j];
}

}  // namespace

template <int TM>
__global__ void __launch_bounds__(FA_THREADS) fa_falsify_kernel(NetDesc net, FalsifyArgs a, RegNetCfg cfg) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, col = lane & 15, grp = lane >> 4;
  const int n0 = net.dims[0];
  const int p = blockIdx.x;
  const int64_t pid = a.pids[p];
  const FalsifyLds L = fa_falsify_lds(a, n0, cfg.floats);
  float* z0 = smem + L.z0;
  float* fm = smem + L.fm;
  int* fq = (int*)(smem + L.fq);
  float* zs = smem + L.zs;
  float* s_lo = smem + L.slo;
  float* s_hi = smem + L.shi;
  int* misc = (int*)(smem + L.misc);        // [0] best flip key, [1] hit, [2] hit j, [3] hit q, [4] change
  const int nl = min(a.n_local, a.n_samples);
  const int V = a.V, Pp = a.Pp;
  const bool rx = fa_fals_relaxed(a);
  const int RV = rx ? 2 * V : V;
  fa_stage_wperm(net, a.flat, smem, tid, FA_THREADS);
  for (int i = tid; i < n0; i += FA_THREADS) {
    s_lo[i] = a.lo[(size_t)p * n0 + i];
    s_hi[i] = a.hi[(size_t)p * n0 + i];
  }
  if (tid == 0) {
    misc[0] = INT_MAX;
    misc[1] = 0;
  }
  __syncthreads();
  float HA[TM][4], HB[TM][4];
  // ================= phase 1: heavy sampling
  for (int r0 = 0; r0 < a.n_samples; r0 += 64) {
    const int s = r0 + wave * 16 + col;
    const bool sv = s < a.n_samples;
    float Xb[TM][4];
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = 16 * t + 4 * grp + i;
        Xb[t][i] = (k < n0 && sv) ? fa_coord(a.seed, pid, s, k, s_lo[k], s_hi[k]) : 0.f;
      }
    for (int v2 = 0; v2 < RV; ++v2) {
      const int v = v2 < V ? v2 : v2 - V;
      const bool xp = v2 >= V;                   // an x' row (relaxed): RA dims shifted
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = 16 * t + 4 * grp + i;
          const int m = k < n0 ? fa_pa_slot(a, k) : -1;
          float val = m >= 0 ? (float)a.values[v * a.npa + m] : Xb[t][i];
          if (xp && k < n0 && sv) {
            const int r = fa_ra_slot(a, k);
            if (r >= 0) val += fa_roff(a, pid, s, r);
          }
          HA[t][i] = val;
        }
      const float z = fa_reg_forward<TM>(net, cfg, smem, lane, HA, HB);
      if (grp == 0) zs[(wave * 16 + col) * RV + v2] = z;   // read back by this same lane only
    }
    if (grp == 0 && sv) {
      const float* zr = zs + (wave * 16 + col) * RV;
      z0[s] = zr[0];
      int gq = 0, fq0 = -1;
      const float g = fa_pair_margin(a, zr, rx, &gq, &fq0);
      if (s < nl) {
        fm[s] = g;
        fq[s] = gq;
      }
      if (fq0 >= 0) atomicMin(&misc[0], s * Pp + fq0);
    }
    __syncthreads();
    if (misc[0] != INT_MAX) break;                 // uniform
  }
  const int key = misc[0];
  if (key != INT_MAX) {
    const int s = key / Pp, q = key % Pp;
    const int vi = (int)a.pairs[2 * q], vj = (int)a.pairs[2 * q + 1];
    for (int d = tid; d < n0; d += FA_THREADS) {
      const float base = fa_coord(a.seed, pid, s, d, s_lo[d], s_hi[d]);
      const int m = fa_pa_slot(a, d);
      const int r = rx ? fa_ra_slot(a, d) : -1;
      a.wit_x[(size_t)p * n0 + d] = m >= 0 ? (float)a.values[vi * a.npa + m] : base;
      a.wit_xp[(size_t)p * n0 + d] = m >= 0 ? (float)a.values[vj * a.npa + m] : base + (r >= 0 ? fa_roff(a, pid, s, r) : 0.f);
    }
    if (tid == 0) {
      a.found[p] = 1;
      a.how[p] = 1;
    }
    return;
  }
  // ================= phase 2: boundary walk between the most positive and most negative samples
  const int kw = min(a.walk_k, a.n_samples);
  if (kw > 0 && a.walk_steps > 0) {
    float* wa = smem + L.wa;
    float* wb = smem + L.wb;
    float* tlo = smem + L.tlo;
    float* thi = smem + L.thi;
    int* wok = (int*)(smem + L.wok);
    int* widx = (int*)(smem + L.widx);
    float* sval = smem + L.sval;
    if (wave == 0) {
      fa_select_extremes(z0, a.n_samples, kw, 1.f, widx, sval, lane);
      fa_select_extremes(z0, a.n_samples, kw, -1.f, widx + kw, sval, lane);
    }
    __syncthreads();
    for (int e = tid; e < kw * n0; e += FA_THREADS) {
      const int j = e / n0, d = e - j * n0;
      wa[e] = fa_coord(a.seed, pid, widx[j], d, s_lo[d], s_hi[d]);
      wb[e] = fa_coord(a.seed, pid, widx[kw + j], d, s_lo[d], s_hi[d]);
    }
    for (int j = tid; j < kw; j += FA_THREADS) {
      wok[j] = (z0[widx[j]] > 0.f) && (z0[widx[kw + j]] < 0.f);
      tlo[j] = 0.f;
      thi[j] = 1.f;
    }
    __syncthreads();
    const int rows = kw * V;
    for (int st = 0; st < a.walk_steps; ++st) {
      for (int g0 = wave * 16; g0 < rows; g0 += 64) {
        const int r = g0 + col;
        const bool rv = r < rows;
        const int j = rv ? r / V : 0, v = rv ? r - (r / V) * V : 0;
        const float tm = 0.5f * (tlo[j] + thi[j]);
#pragma unroll
        for (int t = 0; t < TM; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int k = 16 * t + 4 * grp + i;
            float val = 0.f;
            if (rv && k < n0) {
              const int m = fa_pa_slot(a, k);
              const float A = wa[j * n0 + k], B = wb[j * n0 + k];
              val = m >= 0 ? (float)a.values[v * a.npa + m] : rintf(__fadd_rn(A, __fmul_rn(tm, __fsub_rn(B, A))));
            }
            HA[t][i] = val;
          }
        const float z = fa_reg_forward<TM>(net, cfg, smem, lane, HA, HB);
        if (grp == 0 && rv) zs[r] = z;
      }
      __syncthreads();
      if (tid == 0) {
        int hit = 0, hj = 0, hq = 0;
        for (int j = 0; j < kw && !hit; ++j) {
          if (!wok[j]) continue;
          for (int q = 0; q < Pp; ++q) {
            const float zi = zs[j * V + (int)a.pairs[2 * q]], zj = zs[j * V + (int)a.pairs[2 * q + 1]];
            if ((zi < 0.f && zj > 0.f) || (zi > 0.f && zj < 0.f)) {
              hit = 1; hj = j; hq = q;
              break;
            }
          }
        }
        misc[1] = hit; misc[2] = hj; misc[3] = hq;
      }
      __syncthreads();
      if (misc[1]) {
        const int j = misc[2], q = misc[3];
        const int vi = (int)a.pairs[2 * q], vj = (int)a.pairs[2 * q + 1];
        const float tm = 0.5f * (tlo[j] + thi[j]);
        for (int d = tid; d < n0; d += FA_THREADS) {
          const float A = wa[j * n0 + d], B = wb[j * n0 + d];
          const float base = rintf(__fadd_rn(A, __fmul_rn(tm, __fsub_rn(B, A))));
          const int m = fa_pa_slot(a, d);
          a.wit_x[(size_t)p * n0 + d] = m >= 0 ? (float)a.values[vi * a.npa + m] : base;
          a.wit_xp[(size_t)p * n0 + d] = m >= 0 ? (float)a.values[vj * a.npa + m] : base;
        }
        if (tid == 0) {
          a.found[p] = 1;
          a.how[p] = 2;
        }
        return;
      }
      for (int j = tid; j < kw; j += FA_THREADS) {
        const float tm = 0.5f * (tlo[j] + thi[j]);
        if (zs[j * V] > 0.f) tlo[j] = tm;
        else thi[j] = tm;
      }
      __syncthreads();
    }
  }
  // ================= phase 3: coordinate ascent from the K best-margin samples
  const int K = min(a.K, nl);
  const int nmf = 2 * a.nfree;                   // +-1 on the free dims, then (relaxed) +-1 on the offsets
  const int nm = nmf + (rx ? 2 * a.nra : 0);
  if (K > 0 && nm > 0 && a.iters > 0) {
    float* X = smem + L.X;
    float* F = smem + L.F;
    int* Q = (int*)(smem + L.Q);
    float* marg = smem + L.marg;
    int* margq = (int*)(smem + L.margq);
    float* DK = smem + L.DK;                     // [K, nra] RA offsets of the starts (relaxed)
    int* sidx = (int*)(smem + L.widx);           // the walk is over: reuse its selection slots
    if (wave == 0) fa_select_extremes(fm, nl, K, 1.f, sidx, smem + L.sval, lane);
    __syncthreads();
    for (int e = tid; e < K * n0; e += FA_THREADS) {
      const int j = e / n0, d = e - j * n0;
      X[e] = fa_coord(a.seed, pid, sidx[j], d, s_lo[d], s_hi[d]);
    }
    if (rx)
      for (int e = tid; e < K * a.nra; e += FA_THREADS) {
        const int j = e / a.nra, m = e - j * a.nra;
        DK[e] = fa_roff(a, pid, sidx[j], m);
      }
    for (int j = tid; j < K; j += FA_THREADS) {
      F[j] = fm[sidx[j]];
      Q[j] = fq[sidx[j]];
    }
    __syncthreads();
    const int per = nm * RV, total = K * per;
    for (int it = 0; it < a.iters; ++it) {
      if (tid == 0) {
        int h = 0;
        for (int s = 0; s < K; ++s) h |= F[s] > 0.f;
        misc[1] = h;
        misc[4] = 0;
      }
      __syncthreads();
      if (misc[1]) break;                         // uniform
      for (int g0 = wave * 16; g0 < total; g0 += 64) {
        const int r = g0 + col;
        const bool rv = r < total;
        const int v2 = rv ? r % RV : 0, mv = rv ? (r / RV) % nm : 0, s = rv ? r / per : 0;
        const int v = v2 < V ? v2 : v2 - V;
        const bool xpr = v2 >= V;
        const int fd = mv < nmf ? a.free_idx[mv >> 1] : -1;
        const int rm = mv < nmf ? -1 : (mv - nmf) >> 1;   // RA offset moved by this move
        const float step = (mv & 1) ? 1.f : -1.f;
#pragma unroll
        for (int t = 0; t < TM; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int k = 16 * t + 4 * grp + i;
            float val = 0.f;
            if (rv && k < n0) {
              val = X[s * n0 + k];
              if (k == fd) val = fminf(fmaxf(val + step, s_lo[k]), s_hi[k]);
              if (xpr) {
                const int ro = fa_ra_slot(a, k);
                if (ro >= 0) {
                  float dd = DK[s * a.nra + ro];
                  if (ro == rm) dd = fminf(fmaxf(dd + step, -(float)a.tau), (float)a.tau);
                  val += dd;
                }
              }
              const int m = fa_pa_slot(a, k);
              if (m >= 0) val = (float)a.values[v * a.npa + m];
            }
            HA[t][i] = val;
          }
        const float z = fa_reg_forward<TM>(net, cfg, smem, lane, HA, HB);
        if (grp == 0 && rv) zs[r] = z;
      }
      __syncthreads();
      for (int i = tid; i < K * nm; i += FA_THREADS) {   // best pair per (start, move); first on ties
        int gq = 0, fl = -1;
        marg[i] = fa_pair_margin(a, zs + (size_t)i * RV, rx, &gq, &fl);
        margq[i] = gq;
      }
      __syncthreads();
      for (int s = tid; s < K; s += FA_THREADS) {        // best improving move per start
        float g = -INFINITY;
        int gm = 0;
        for (int mv = 0; mv < nm; ++mv)
          if (marg[s * nm + mv] > g) { g = marg[s * nm + mv]; gm = mv; }
        if (g > F[s]) {
          const float step = (gm & 1) ? 1.f : -1.f;
          if (gm < nmf) {
            const int d = a.free_idx[gm >> 1];
            X[s * n0 + d] = fminf(fmaxf(X[s * n0 + d] + step, s_lo[d]), s_hi[d]);
          } else {
            float& dd = DK[s * a.nra + ((gm - nmf) >> 1)];
            dd = fminf(fmaxf(dd + step, -(float)a.tau), (float)a.tau);
          }
          F[s] = g;
          Q[s] = margq[s * nm + gm];
          misc[4] = 1;
        }
      }
      __syncthreads();
      if (!misc[4]) break;
      __syncthreads();
    }
    __syncthreads();
    int sh = -1;
    for (int s = 0; s < K; ++s)
      if (F[s] > 0.f) { sh = s; break; }
    if (sh >= 0) {
      const int q = Q[sh];
      const int vi = (int)a.pairs[2 * q], vj = (int)a.pairs[2 * q + 1];
      for (int d = tid; d < n0; d += FA_THREADS) {
        const int m = fa_pa_slot(a, d);
        const int ro = rx ? fa_ra_slot(a, d) : -1;
        const float x = X[sh * n0 + d];
        a.wit_x[(size_t)p * n0 + d] = m >= 0 ? (float)a.values[vi * a.npa + m] : x;
        a.wit_xp[(size_t)p * n0 + d] = m >= 0 ? (float)a.values[vj * a.npa + m] : x + (ro >= 0 ? DK[sh * a.nra + ro] : 0.f);
      }
      if (tid == 0) {
        a.found[p] = 1;
        a.how[p] = 3;
      }
      return;
    }
  }
  if (tid == 0) {
    a.found[p] = 0;
    a.how[p] = 0;
  }
}

namespace {
typedef void (*FalsifyKernel)(NetDesc, FalsifyArgs, RegNetCfg);
FalsifyKernel select_falsify(int TM) {
  if (TM <= 1) return fa_falsify_kernel<1>;
  if (TM <= 2) return fa_falsify_kernel<2>;
  if (TM <= 4) return fa_falsify_kernel<4>;
  if (TM <= 7) return fa_falsify_kernel<7>;
  return nullptr;
}
}  // namespace

// 1 launched, 0 unsupported shape (the caller keeps the PyTorch path), < 0 bad arguments.
extern "C" int fa_falsify_launch(const NetDesc& net, FalsifyArgs a, hipStream_t stream) {
  if (a.P <= 0) return 1;
  if (a.npa > FA_MAX_PA || a.nfree > 64 || a.V <= 0 || a.Pp <= 0 || a.n_samples <= 0 || a.K < 0 ||
      a.walk_k < 0 || a.n_local < 0 || a.nra < 0 || a.nra > FA_MAX_RA || a.tau < 0)
    return -3;
  if ((long long)a.n_samples * a.Pp >= INT_MAX) return -3;   // flip keys sample * Pp + pair are int
  FalsifyKernel k = select_falsify(fa_regnet_tm(net));
  if (!k) return 0;
  RegNetCfg cfg{};
  if (!fa_regnet_cfg(net, cfg)) return -1;
  const FalsifyLds L = fa_falsify_lds(a, net.dims[0], cfg.floats);
  const size_t bytes = (size_t)L.floats * sizeof(float);
  if (bytes > 160 * 1024) return 0;
  if (!fa_lds_ok(bytes)) return -4;
  hipLaunchKernelGGL(k, dim3((unsigned)a.P), dim3(FA_THREADS), bytes, stream, net, a, cfg);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 1 : -(int)e;
}

FA_LDS_REGISTER(FA_LDS_K(fa_falsify_kernel<1>), FA_LDS_K(fa_falsify_kernel<2>), FA_LDS_K(fa_falsify_kernel<4>),
                FA_LDS_K(fa_falsify_kernel<7>));
