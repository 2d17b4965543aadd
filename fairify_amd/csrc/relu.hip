// ReLU-phase branch-and-bound kernels (stage "relu", engine/relu_bab.py).  gfx950.
//
// The residue of the input-split search on zero-bias narrow nets is dominated by EXACT zeros:
// the logit is 0 on a region where every path to it is dead, and the strict query N(x) < 0 <
// N(x') needs bounds that reach 0 exactly.  A node here is (partition, ordered PA pair, input
// box, phase of every hidden neuron of the two network copies); its rows 2n / 2n+1 are the copies
// that must be < 0 / > 0.
//
// fa_crown_phase_kernel  backward (CROWN) bounds of the logit per row and sign, for three lower-
//                        slope policies, concretised at EVERY layer before it is relaxed and at
//                        the input box; coefficient rounding is carried as per-coefficient
//                        intervals [lambda - E, lambda + E] (charged to the constant only where
//                        the sign is uncertain), so a term whose range starts at 0 with a
//                        certainly non-negative coefficient contributes exactly 0.  Emits the
//                        neuron whose chord intercept the best bound pays most (branching).
//                        Same arithmetic as ops/reference.py:crown_phase.
// fa_relu_rows_kernel    node boxes -> row boxes (PA dims set per row), per-partition node counts
// fa_relu_cert_kernel    sign shortcut (copy 0 >= 0 or copy 1 <= 0 on the branch region, empty
//                        region), else the coupled certificate min_t max_x t(-L_A) + (1-t) U_B;
//                        open nodes get their LP-optimal vertex pair and a branching decision
// fa_relu_split_kernel   candidate pairs to the host check, children (ReLU phase or input halves)
// fa_relu_settle_kernel  level end: STOPPING -> UNKNOWN, counters to pinned host memory
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>

#include "args.h"

#define ST_UNKNOWN 0
#define ST_RUNNING 3
#define ST_STOPPING 4

__device__ __forceinline__ float fa_gamr(int k, float u) {
  const float ku = (float)(k + 2) * u;
  return ku / (1.f - ku) * (1.f + 4.f * u);
}

template <int G>
__device__ __forceinline__ float fa_gsum(float v) {
#pragma unroll
  for (int off = G / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// (score, index) arg-max within a group; ties -> lower index
template <int G>
__device__ __forceinline__ void fa_gargmax(float& s, int& i) {
#pragma unroll
  for (int off = G / 2; off > 0; off >>= 1) {
    const float s2 = __shfl_xor(s, off, 64);
    const int i2 = __shfl_xor(i, off, 64);
    if (s2 > s || (s2 == s && i2 < i)) { s = s2; i = i2; }
  }
}

#define FA_CP_WAVES 4

template <int G>
__global__ void __launch_bounds__(64 * FA_CP_WAVES) fa_crown_phase_kernel(NetDesc net, CrownPhaseArgs a, int nparams,
                                                                          int WP) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int RPW = 64 / G;
  const int tid = threadIdx.x;
  // W_l transposed ([n_out][n_in]) + biases at their `flat` offsets (fa_crown_kernel's layout)
  for (int l = 0; l < net.n_layers; ++l) {
    const int nin = net.dims[l], nout = net.dims[l + 1];
    const float* src = a.flat + net.w_off[l];
    float* dst = smem + net.w_off[l];
    for (int e = tid; e < nin * nout; e += 64 * FA_CP_WAVES) {
      const int j = e / nin, i = e - j * nin;
      dst[e] = src[(size_t)i * nout + j];
    }
    for (int e = tid; e < nout; e += 64 * FA_CP_WAVES) smem[net.b_off[l] + e] = a.flat[net.b_off[l] + e];
  }
  __syncthreads();
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int grp = lane / G;
  const int gl = lane % G;
  float* lam = smem + nparams + (wave * RPW + grp) * (5 * WP + 1);
  float* E = lam + WP;
  float* mu = E + WP;
  float* Emu = mu + WP;
  float* bf = Emu + WP;
  const int L = net.n_layers;
  const int n0 = net.dims[0];
  const int N = net.n_neurons;
  const int nh = net.n_hidden;
  const float u = net.unit;
  int K = 4 * L + 4;
  for (int l = 0; l < L; ++l) K += 2 * net.dims[l + 1];
  const float gK = fa_gamr(K, u);
  const float g0 = fa_gamr(n0 + 1, u);
  const float g1 = fa_gamr(1, u);
  const int rows_per_block = FA_CP_WAVES * RPW;
  for (int rb = blockIdx.x * rows_per_block; rb < a.R; rb += gridDim.x * rows_per_block) {
    const int r0 = rb + wave * RPW + grp;
    bool valid = r0 < a.R;
    const int r = valid ? r0 : a.R - 1;             // idle groups shadow the last row, never write
    if (valid && a.skip_status) {
      const int8_t st = a.skip_status[a.skip_part[r]];
      valid = st == ST_RUNNING || st == ST_STOPPING;
    }
    if (!__any(valid)) continue;                    // wave-uniform
    const int8_t* ph = a.phase ? a.phase + (size_t)r * nh : nullptr;
    const float* lbr = a.layer_lb + (size_t)r * N;
    const float* ubr = a.layer_ub + (size_t)r * N;
    const float fw_lb = a.out_lb[r], fw_ub = a.out_ub[r];
    float res_low[2], res_score[2];
    int res_split[2];
#pragma unroll 1
    for (int si = 0; si < 2; ++si) {
      const float sg = si == 0 ? 1.f : -1.f;
      float best_total = -INFINITY, bscore = -1.f, best_in = -INFINITY, bf_c = 0.f, bf_err = 0.f;
      int bsplit = -1;
#pragma unroll 1
      for (int pol = 0; pol < 3; ++pol) {
        {
          const int n = net.dims[L - 1];
          const float* W = smem + net.w_off[L - 1];        // [1][n]
          for (int j = gl; j < n; j += G) {
            lam[j] = sg * W[j];
            E[j] = 0.f;
          }
        }
        float c = sg * smem[net.b_off[L - 1]], err = 0.f, pol_best = -INFINITY, sc_best = -1.f;
        int sc_idx = -1;
        __builtin_amdgcn_wave_barrier();
#pragma unroll 1
        for (int l = L - 2; l >= 0; --l) {
          const int n = net.dims[l + 1];
          const int nin = net.dims[l];
          const int off = net.neuron_off[l];
          const float* W = smem + net.w_off[l];
          const float* b = smem + net.b_off[l];
          float tsum = 0.f, tmag = 0.f, errc = 0.f, erel = 0.f, cs = 0.f, cm = 0.f, eb = 0.f, lsc = -1.f;
          int lidx = 0x7fffffff;
          for (int j = gl; j < n; j += G) {
            const float lb = lbr[off + j], ub = ubr[off + j];
            const int p = ph ? (int)ph[off + j] : 0;
            const bool dd = ub <= 0.f || p < 0;
            const bool fact = p > 0 && !dd;
            const bool act = lb >= 0.f && !dd;
            const bool unst = !dd && !act;
            const float alo = dd ? 0.f : fmaxf(lb, 0.f);
            const float ahi = dd ? 0.f : fmaxf(ub, 0.f);
            const float lm = lam[j];
            float e = E[j];
            // concretisation at this layer's post-activations
            const bool ex0 = ahi == 0.f || (alo == 0.f && lm - e >= 0.f);
            const float prod = fminf(lm * alo, lm * ahi), ep = e * ahi;
            if (!ex0) {
              tsum += prod - ep;
              tmag += fabsf(prod) + ep;
            }
            // uncertain sign: relax the computed value, charge the interval
            const bool unc = (lm - e < 0.f) && (lm + e > 0.f) && !dd;
            if (unc) errc += e * ahi;
            if (unc || dd) e = 0.f;
            const float alpha = pol == 0 ? (ub > -lb ? 1.f : 0.f) : (pol == 1 ? 0.f : 1.f);
            const bool chord_ok = unst && !fact;
            const float den = ub - lb;
            const float s_ch = chord_ok ? (ub / den) * (1.f + 4.f * u) : 1.f;
            const float slope = act ? 1.f : (dd ? 0.f : (lm >= 0.f ? alpha : s_ch));
            const float m = lm * slope;
            const bool chord = chord_ok && lm < 0.f;
            const float t = chord ? -m * lb : 0.f;
            if (chord) erel += 3.f * u * (fabsf(m) * fmaxf(fabsf(lb), fabsf(ub)) + fabsf(t)) + e * s_ch * fabsf(lb);
            const float emu = e * slope * (1.f + 4.f * u);
            const float bj = b[j];
            cs += m * bj + t;
            cm += fabsf(m * bj) + fabsf(t);
            eb += emu * fabsf(bj);
            mu[j] = m;
            Emu[j] = emu;
            if (chord_ok && p == 0) {
              const float sc = fabsf(t) + 1e-3f * fabsf(lm) * (-ub * lb / den);
              if (sc > lsc || (sc == lsc && off + j < lidx)) { lsc = sc; lidx = off + j; }
            }
          }
          tsum = fa_gsum<G>(tsum);
          tmag = fa_gsum<G>(tmag);
          errc = fa_gsum<G>(errc);
          erel = fa_gsum<G>(erel);
          cs = fa_gsum<G>(cs);
          cm = fa_gsum<G>(cm);
          eb = fa_gsum<G>(eb);
          fa_gargmax<G>(lsc, lidx);
          const float v = (tsum + c) - err * (1.f + 2.f * gK) - fa_gamr(n + 3, u) * (tmag + fabsf(c));
          pol_best = fmaxf(pol_best, v);
          err += errc;
          if (lsc > sc_best) { sc_best = lsc; sc_idx = lidx; }
          const float cold = c;
          c = cold + cs;
          err += erel + fa_gamr(2 * n + 1, u) * (fabsf(cold) + cm) + eb;
          __builtin_amdgcn_wave_barrier();
          const float gn = fa_gamr(n + 1, u);
          for (int i = gl; i < nin; i += G) {
            float acc = 0.f, q1 = 0.f, q2 = 0.f;
            for (int j = 0; j < n; ++j) {
              const float w = W[(size_t)j * nin + i];
              const float mj = mu[j];
              acc = fmaf(w, mj, acc);
              q1 = fmaf(fabsf(w), Emu[j], q1);
              q2 = fmaf(fabsf(w), fabsf(mj), q2);
            }
            lam[i] = acc;
            E[i] = q1 * (1.f + gn) + gn * q2;
          }
          __builtin_amdgcn_wave_barrier();
        }
        // ---- concretise over the input box
        float ein = 0.f, cp = 0.f, mp = 0.f;
        for (int i = gl; i < n0; i += G) {
          const float xl = a.lo[(size_t)r * n0 + i], xh = a.hi[(size_t)r * n0 + i];
          const float lm = lam[i];
          const float mx = fmaxf(fabsf(xl), fabsf(xh));
          ein += E[i] * mx;
          cp += fminf(lm * xl, lm * xh);
          mp += fabsf(lm) * mx;
        }
        ein = fa_gsum<G>(ein);
        cp = fa_gsum<G>(cp);
        mp = fa_gsum<G>(mp);
        const float err_in = (err + ein) * (1.f + 2.f * gK);
        const float conc = cp + c;
        const float cmg = mp + fabsf(c);
        const float low_in = conc - err_in - g0 * cmg - g1 * fabsf(conc);
        pol_best = fmaxf(pol_best, low_in);
        if (pol_best > best_total) {
          best_total = pol_best;
          bsplit = sc_idx;
          bscore = sc_best;
        }
        if (low_in > best_in) {
          best_in = low_in;
          for (int i = gl; i < n0; i += G) bf[i] = lam[i];
          bf_c = c;
          bf_err = err_in;
        }
        __builtin_amdgcn_wave_barrier();
      }
      res_low[si] = best_total;
      res_split[si] = bscore > 0.f ? bsplit : -1;
      res_score[si] = bscore;
      if (valid) {
        if (si == 0 && best_in >= fw_lb) {
          for (int i = gl; i < n0; i += G) a.Lc[(size_t)r * n0 + i] = bf[i];
          if (gl == 0) { a.L0[r] = bf_c; a.Le[r] = bf_err; }
        } else if (si == 1 && -best_in <= fw_ub) {
          for (int i = gl; i < n0; i += G) a.Uc[(size_t)r * n0 + i] = -bf[i];
          if (gl == 0) { a.U0[r] = -bf_c; a.Ue[r] = bf_err; }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (valid && gl == 0) {
      float ol = fmaxf(fw_lb, res_low[0]), ou = fminf(fw_ub, -res_low[1]);
      if (a.infeas && a.infeas[r]) { ol = INFINITY; ou = -INFINITY; }
      a.out_lb[r] = ol;
      a.out_ub[r] = ou;
      a.split[2 * r] = res_split[0];
      a.split[2 * r + 1] = res_split[1];
      a.score[2 * r] = res_score[0];
      a.score[2 * r + 1] = res_score[1];
      if (a.low) { a.low[2 * r] = res_low[0]; a.low[2 * r + 1] = res_low[1]; }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// LDS bytes of fa_crown_phase_kernel for `net`, 0 if it does not fit (a layer wider than 256 or
// more than 160 KB): checked before a ReluRuntime is built (engine/relu_bab.py), so a network the
// kernel cannot hold skips the relu stage instead of aborting a level
extern "C" size_t fa_crown_phase_bytes(const NetDesc& net) {
  int wmax = 1;
  for (int l = 0; l <= net.n_layers; ++l) {
    if (net.dims[l] > 256) return 0;
    if (l > 0) wmax = std::max(wmax, net.dims[l]);
  }
  int G = 4;
  while (G < wmax && G < 64) G *= 2;
  const int WP = (std::max(wmax, net.dims[0]) + 3) & ~3;
  const int nparams = net.b_off[net.n_layers - 1] + net.dims[net.n_layers];
  const int rows_per_block = FA_CP_WAVES * (64 / G);
  const size_t bytes = ((size_t)nparams + (size_t)rows_per_block * (5 * WP + 1)) * sizeof(float);
  return bytes > 160 * 1024 ? 0 : bytes;
}

// 0 launched, -1 the network does not fit (layer wider than 256 or LDS), < -1 launch error
extern "C" int fa_crown_phase_launch(const NetDesc& net, CrownPhaseArgs a, hipStream_t stream) {
  if (a.R <= 0) return 0;
  if (fa_crown_phase_bytes(net) == 0) return -1;
  int wmax = 1;
  for (int l = 0; l <= net.n_layers; ++l) {
    if (net.dims[l] > 256) return -1;
    if (l > 0) wmax = std::max(wmax, net.dims[l]);
  }
  int G = 4;
  while (G < wmax && G < 64) G *= 2;
  const int WP = (std::max(wmax, net.dims[0]) + 3) & ~3;
  const int nparams = net.b_off[net.n_layers - 1] + net.dims[net.n_layers];
  const int rows_per_block = FA_CP_WAVES * (64 / G);
  const size_t bytes = ((size_t)nparams + (size_t)rows_per_block * (5 * WP + 1)) * sizeof(float);
  if (bytes > 160 * 1024) return -1;
  typedef void (*K)(NetDesc, CrownPhaseArgs, int, int);
  K k = G == 4 ? fa_crown_phase_kernel<4> : G == 8 ? fa_crown_phase_kernel<8> : G == 16 ? fa_crown_phase_kernel<16>
      : G == 32 ? fa_crown_phase_kernel<32> : fa_crown_phase_kernel<64>;
  if (!fa_lds_ok(bytes)) return -3;
  const int blocks = (int)std::min<long long>(((long long)a.R + rows_per_block - 1) / rows_per_block, 256LL * 8);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(64 * FA_CP_WAVES), bytes, stream, net, a, nparams, WP);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e - 10;
}

// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int fa_pa_slot(const ReluLevelArgs& a, int d) {
  for (int k = 0; k < a.npa; ++k)
    if (a.pa_idx[k] == d) return k;
  return -1;
}

__global__ void fa_relu_rows_kernel(ReluLevelArgs a) {
  const long long tot = 2LL * a.Nn * a.n0;
  for (long long e = (long long)blockIdx.x * FA_THREADS + threadIdx.x; e < tot; e += (long long)gridDim.x * FA_THREADS) {
    const int row = (int)(e / a.n0), d = (int)(e - (long long)row * a.n0);
    const int n = row >> 1, side = row & 1;
    // relaxed: copy B reads x''s box on the RA dims; every other dim is shared with x, and only x's box
    // follows the input splits there (the x' box keeps its root values off the RA dims)
    bool xp = false;
    if (a.nra > 0 && side == 1)
      for (int k = 0; k < a.nra; ++k) xp = xp || a.ra_idx[k] == d;
    float lo = (xp ? a.xplo : a.xlo)[(size_t)n * a.n0 + d], hi = (xp ? a.xphi : a.xhi)[(size_t)n * a.n0 + d];
    const int k = fa_pa_slot(a, d);
    if (k >= 0) {
      const int v = (int)a.pairs[2 * a.pair[n] + side];
      lo = hi = a.values[v * a.npa + k];
    }
    a.rlo[e] = lo;
    a.rhi[e] = hi;
    if (d == 0) {
      const int p = a.part[n];
      a.rpart[row] = p;
      if (side == 0) atomicAdd(&a.part_nodes[p], 1);
    }
  }
}

// One thread per node.  NM >= n0 (register arrays).  RX: relaxed query (a.nra > 0; the PA-only
// instance keeps its registers: the x' arrays fold away)
template <int NM, bool RX>
__global__ void __launch_bounds__(FA_THREADS) fa_relu_cert_kernel(ReluLevelArgs a) {
  const int n = blockIdx.x * FA_THREADS + threadIdx.x;
  if (n >= a.Nn) return;
  const int n0 = a.n0;
  const int A = 2 * n, B = 2 * n + 1;
  const int p = a.part[n];
  uint8_t open = 0;
  int choice = -3, idim = -1;
  const int8_t st = a.status[p];
  // relaxed: x_r and x'_r boxes more than tau apart leave no admissible pair -- the node is closed
  bool admissible = true;
  for (int m = 0; RX && m < a.nra; ++m) {
    const int d = a.ra_idx[m];
    const size_t o = (size_t)n * n0 + d;
    if (a.xplo[o] > a.xhi[o] + a.tau || a.xphi[o] < a.xlo[o] - a.tau) admissible = false;
  }
  // orientation -1 (pair >= neg_from): N(x, va) > 0 > N(x', vb) is N_A' < 0 < N_B' on the negated
  // logit, whose lower form is -U and upper form -L: copy A's U forms / copy B's L forms, negated
  const bool ng = a.neg_from > 0 && a.pair[n] >= a.neg_from;
  const float lbA = ng ? -a.oub[A] : a.olb[A], ubB = ng ? -a.olb[B] : a.oub[B];
  if ((st == ST_RUNNING || st == ST_STOPPING) && admissible && !(a.infeas[A] || a.infeas[B]) &&
      !(lbA >= 0.f) && !(ubB <= 0.f)) {
    const int vA = (int)a.pairs[2 * a.pair[n]], vB = (int)a.pairs[2 * a.pair[n] + 1];
    float ca[NM], cb[NM], xl[NM], xh[NM], pl[NM], ph[NM];
    bool rd[NM];                         // relaxed: RA dim (copies concretised separately)
    float fA = 0.f, fB = 0.f;
    float fmA = 0.f, fmB = 0.f;          // sum |ca_i v_k|: the folded products' rounding magnitude
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      const bool v = i < n0;
      ca[i] = v ? (ng ? -a.Uc[(size_t)A * n0 + i] : a.Lc[(size_t)A * n0 + i]) : 0.f;
      cb[i] = v ? (ng ? -a.Lc[(size_t)B * n0 + i] : a.Uc[(size_t)B * n0 + i]) : 0.f;
      xl[i] = v ? a.xlo[(size_t)n * n0 + i] : 0.f;
      xh[i] = v ? a.xhi[(size_t)n * n0 + i] : 0.f;
      bool r = false;
      for (int m = 0; RX && m < a.nra; ++m) r = r || a.ra_idx[m] == i;
      rd[i] = RX && v && r;
      if (RX) {
        pl[i] = rd[i] ? a.xplo[(size_t)n * n0 + i] : xl[i];
        ph[i] = rd[i] ? a.xphi[(size_t)n * n0 + i] : xh[i];
      }
    }
    for (int k = 0; k < a.npa; ++k) {   // fold the PA coordinates (fixed per row) into the constants
      const int d = a.pa_idx[k];
#pragma unroll
      for (int i = 0; i < NM; ++i)
        if (i == d) {
          fA += ca[i] * a.values[vA * a.npa + k];
          fB += cb[i] * a.values[vB * a.npa + k];
          fmA += fabsf(ca[i] * a.values[vA * a.npa + k]);
          fmB += fabsf(cb[i] * a.values[vB * a.npa + k]);
          ca[i] = cb[i] = 0.f;
          xl[i] = xh[i] = 0.f;
          if (RX) pl[i] = ph[i] = 0.f;
        }
    }
    // lower constant of copy A's (oriented) logit less its error; upper constant of copy B's plus its error
    const float LA0 = ng ? -(a.U0[A] + a.Ue[A]) : a.L0[A] - a.Le[A];
    const float UB0 = ng ? -(a.L0[B] - a.Le[B]) : a.U0[B] + a.Ue[B];
    // with several PA dims the folded sum can cancel: the margin takes the terms' magnitudes
    float magA = fabsf(LA0) + fmA, magB = fabsf(UB0) + fmB;
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      const float mx = fmaxf(fabsf(xl[i]), fabsf(xh[i]));
      const float mxb = RX ? fmaxf(fabsf(pl[i]), fabsf(ph[i])) : mx;   // copy B's box (x' on RA dims)
      magA += fabsf(ca[i]) * mx;
      magB += fabsf(cb[i]) * mxb;
      ca[i] = -ca[i];                      // A = -L_A
    }
    const float A0 = -(LA0 + fA), B0 = UB0 + fB;
    const float marg0 = 8.f * a.unit * (magA + magB);
    auto g_at = [&](float t) {
      float val = 0.f;
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        if (RX && rd[i]) {   // x_r and x'_r concretised separately (the tie only loosens when dropped)
          const float ar = t * ca[i], br = (1.f - t) * cb[i];
          val += fmaxf(ar * xl[i], ar * xh[i]) + fmaxf(br * pl[i], br * ph[i]);
        } else {
          const float cs = t * ca[i] + (1.f - t) * cb[i];
          val += fmaxf(cs * xl[i], cs * xh[i]);
        }
      }
      return val + t * A0 + (1.f - t) * B0 + a.gmarg * (t * magA + (1.f - t) * magB) + marg0;
    };
    float best = g_at(0.f), bt = 0.f;
    {
      const float g1 = g_at(1.f);
      if (g1 < best) { best = g1; bt = 1.f; }
    }
#pragma unroll 1
    for (int i = 0; i < n0; ++i) {
      float ai = 0.f, bi = 0.f;
      bool ri = false;
#pragma unroll
      for (int k = 0; k < NM; ++k)
        if (k == i) { ai = ca[k]; bi = cb[k]; ri = RX && rd[k]; }
      if (ri) continue;                    // separate linear terms in t: no interior breakpoint
      const float den = ai - bi;
      if (den == 0.f) continue;
      const float t = -bi / den;
      if (!(t > 0.f && t < 1.f)) continue;
      const float g = g_at(t);
      if (g < best) { best = g; bt = t; }
    }
    if (!(best <= 0.f)) {                 // NaN keeps the node open
      open = 1;
      float bs = -1.f;
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        if (i >= n0) break;
        const float c = bt * ca[i] + (1.f - bt) * cb[i];
        const float x = c > 0.f ? a.xhi[(size_t)n * n0 + i] : a.xlo[(size_t)n * n0 + i];
        const int k = fa_pa_slot(a, i);
        if (RX && rd[i]) {
          // relaxed RA dim: x_r at copy A's vertex, x'_r at copy B's, pulled into [x_r - tau, x_r + tau]
          const float xa = ca[i] > 0.f ? a.xhi[(size_t)n * n0 + i] : a.xlo[(size_t)n * n0 + i];
          const float xb0 = cb[i] > 0.f ? a.xphi[(size_t)n * n0 + i] : a.xplo[(size_t)n * n0 + i];
          a.cpts[(size_t)A * n0 + i] = xa;
          a.cpts[(size_t)B * n0 + i] = fminf(fmaxf(xb0, xa - a.tau), xa + a.tau);
          // input-split scores: x's dim by copy A's coefficient, x''s by copy B's (idim >= n0)
          const float w = xh[i] - xl[i], wp = ph[i] - pl[i];
          if (w > 0.f) {
            const float s = fabsf(bt * ca[i]) * w + 1e-9f * w;
            if (s > bs) { bs = s; idim = i; }
          }
          if (wp > 0.f) {
            const float s = fabsf((1.f - bt) * cb[i]) * wp + 1e-9f * wp;
            if (s > bs) { bs = s; idim = n0 + i; }
          }
          continue;
        }
        a.cpts[(size_t)A * n0 + i] = k >= 0 ? a.values[vA * a.npa + k] : x;
        a.cpts[(size_t)B * n0 + i] = k >= 0 ? a.values[vB * a.npa + k] : x;
        const float w = xh[i] - xl[i];
        if (k < 0 && w > 0.f) {
          const float s = fabsf(c) * w + 1e-9f * w;
          if (s > bs) { bs = s; idim = i; }
        }
      }
      if (idim < 0) {
        choice = -2;                       // single lattice point: decided by the exact check
      } else {
        // the bound closest to closing and its split: copy A's lower (oriented) bound, copy B's upper
        const float gapA = -lbA, gapB = ubB;
        const int sA = a.split[2 * A + (ng ? 1 : 0)], sB = a.split[2 * B + (ng ? 0 : 1)];
        const bool useA = sA >= 0 && (gapA <= gapB || sB < 0);
        const bool useB = !useA && sB >= 0;
        choice = useA ? sA : (useB ? 65536 + sB : -1);
      }
    }
  }
  a.open[n] = open;
  a.choice[n] = choice;
  a.idim[n] = idim;
}

// One wave64 per node (grid-stride).
__global__ void __launch_bounds__(FA_THREADS) fa_relu_split_kernel(ReluLevelArgs a) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int n0 = a.n0;
  const int w2 = 2 * a.nh;
  for (int n = blockIdx.x * (FA_THREADS / 64) + wave; n < a.Nn; n += gridDim.x * (FA_THREADS / 64)) {
    if (!a.open[n]) continue;                                   // wave-uniform
    const int p = a.part[n];
    const int8_t st = a.status[p];
    if (st != ST_RUNNING && st != ST_STOPPING) continue;
    // ---- the LP-optimal vertex pair, if its rigorous point bounds allow a violation (of this node's
    // orientation)
    const bool ng = a.neg_from > 0 && a.pair[n] >= a.neg_from;
    const bool poss = ng ? (a.pe_ub[2 * n] > 0.f && a.pe_lb[2 * n + 1] < 0.f)
                         : (a.pe_lb[2 * n] < 0.f && a.pe_ub[2 * n + 1] > 0.f);
    if (poss) {
      int slot = 0;
      if (lane == 0) slot = atomicAdd(a.cand_count, 1);
      slot = __shfl(slot, 0);
      if (slot < a.cand_cap) {
        float* cb = a.cand_buf + (size_t)slot * (2 * n0 + 1);
        for (int d = lane; d < 2 * n0 + 1; d += 64)
          cb[d] = d < n0 ? a.cpts[(size_t)(2 * n) * n0 + d]
                         : (d < 2 * n0 ? a.cpts[(size_t)(2 * n + 1) * n0 + d - n0] : __int_as_float(p));
      } else if (lane == 0) {
        a.status[p] = ST_STOPPING;                               // cannot confirm: stay sound
      }
    }
    const int ch = a.choice[n];
    if (ch == -2 || ch == -3) continue;                          // leaf: the exact check decides
    if (st == ST_STOPPING || a.nodes_start[p] >= a.budget) {
      if (lane == 0) a.status[p] = ST_STOPPING;
      continue;
    }
    int off = 0;
    if (lane == 0) off = atomicAdd(a.count_out, 2);
    off = __shfl(off, 0);
    if (off + 2 > a.cap) {
      if (lane == 0) a.status[p] = ST_STOPPING;
      continue;
    }
    if (lane < 2) {
      a.opart[off + lane] = p;
      a.opair[off + lane] = a.pair[n];
    }
    const int dsplit = ch == -1 ? a.idim[n] : -1;    // >= n0: x''s RA dim dsplit - n0 (relaxed)
    for (int e = lane; e < 2 * n0; e += 64) {
      const int c = e / n0, d = e - c * n0;
      float lo = a.xlo[(size_t)n * n0 + d], hi = a.xhi[(size_t)n * n0 + d];
      if (d == dsplit) {
        const float mid = floorf(0.5f * (lo + hi));
        if (c == 0) hi = mid; else lo = mid + 1.f;
      }
      a.oxlo[(size_t)(off + c) * n0 + d] = lo;
      a.oxhi[(size_t)(off + c) * n0 + d] = hi;
      if (a.nra > 0) {
        float plo = a.xplo[(size_t)n * n0 + d], phi = a.xphi[(size_t)n * n0 + d];
        if (d + n0 == dsplit) {
          const float mid = floorf(0.5f * (plo + phi));
          if (c == 0) phi = mid; else plo = mid + 1.f;
        }
        a.oxplo[(size_t)(off + c) * n0 + d] = plo;
        a.oxphi[(size_t)(off + c) * n0 + d] = phi;
      }
    }
    const int kfix = ch >= 0 ? (ch >> 16) * a.nh + (ch & 0xffff) : -1;
    for (int e = lane; e < 2 * w2; e += 64) {
      const int c = e / w2, k = e - c * w2;
      int8_t v = a.phase[(size_t)n * w2 + k];
      if (k == kfix) v = c == 0 ? (int8_t)-1 : (int8_t)1;
      a.ophase[(size_t)(off + c) * w2 + k] = v;
    }
  }
}

__global__ void fa_relu_settle_kernel(int P, int8_t* status, const int* part_nodes, int* nodes_start,
                                      int* counters, int* host_counts) {
  const int p = blockIdx.x * FA_THREADS + threadIdx.x;
  if (p == 0) {
    __hip_atomic_store(&host_counts[0], counters[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&host_counts[1], counters[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (p >= P) return;
  if (status[p] == ST_STOPPING) status[p] = ST_UNKNOWN;
  nodes_start[p] = part_nodes[p];
}

__global__ void fa_relu_reset_kernel(int* counters) {
  if (threadIdx.x < 2) counters[threadIdx.x] = 0;
}

extern "C" int fa_relu_rows_launch(ReluLevelArgs a, hipStream_t stream) {
  if (a.Nn <= 0) return 0;
  if (a.npa > FA_CMAX_PA) return -3;
  const long long tot = 2LL * a.Nn * a.n0;
  const int blocks = (int)std::min<long long>((tot + FA_THREADS - 1) / FA_THREADS, 8192);
  hipLaunchKernelGGL(fa_relu_rows_kernel, dim3(blocks), dim3(FA_THREADS), 0, stream, a);
  return (int)hipGetLastError();
}

extern "C" int fa_relu_cert_launch(ReluLevelArgs a, hipStream_t stream) {
  if (a.Nn <= 0) return 0;
  const dim3 g((a.Nn + FA_THREADS - 1) / FA_THREADS);
  const bool rx = a.nra > 0;
  if (a.n0 <= 16) {
    if (rx) hipLaunchKernelGGL((fa_relu_cert_kernel<16, true>), g, dim3(FA_THREADS), 0, stream, a);
    else hipLaunchKernelGGL((fa_relu_cert_kernel<16, false>), g, dim3(FA_THREADS), 0, stream, a);
  } else if (a.n0 <= 32) {
    if (rx) hipLaunchKernelGGL((fa_relu_cert_kernel<32, true>), g, dim3(FA_THREADS), 0, stream, a);
    else hipLaunchKernelGGL((fa_relu_cert_kernel<32, false>), g, dim3(FA_THREADS), 0, stream, a);
  } else if (a.n0 <= 64) {
    if (rx) hipLaunchKernelGGL((fa_relu_cert_kernel<64, true>), g, dim3(FA_THREADS), 0, stream, a);
    else hipLaunchKernelGGL((fa_relu_cert_kernel<64, false>), g, dim3(FA_THREADS), 0, stream, a);
  }
  else return -4;
  return (int)hipGetLastError();
}

extern "C" int fa_relu_split_launch(ReluLevelArgs a, hipStream_t stream) {
  if (a.Nn <= 0) return 0;
  const int blocks = (int)std::min<long long>(((long long)a.Nn + 3) / 4, 8192);
  hipLaunchKernelGGL(fa_relu_split_kernel, dim3(blocks), dim3(FA_THREADS), 0, stream, a);
  return (int)hipGetLastError();
}

extern "C" int fa_relu_settle_launch(int P, int8_t* status, const int* part_nodes, int* nodes_start, int* counters,
                                     int* host_counts, hipStream_t stream) {
  const int n = P > 0 ? P : 1;
  hipLaunchKernelGGL(fa_relu_settle_kernel, dim3((n + FA_THREADS - 1) / FA_THREADS), dim3(FA_THREADS), 0, stream, P,
                     status, part_nodes, nodes_start, counters, host_counts);
  return (int)hipGetLastError();
}

extern "C" int fa_relu_reset_launch(int* counters, hipStream_t stream) {
  hipLaunchKernelGGL(fa_relu_reset_kernel, dim3(1), dim3(64), 0, stream, counters);
  return (int)hipGetLastError();
}

FA_LDS_REGISTER(FA_LDS_K(fa_crown_phase_kernel<4>), FA_LDS_K(fa_crown_phase_kernel<8>),
                FA_LDS_K(fa_crown_phase_kernel<16>), FA_LDS_K(fa_crown_phase_kernel<32>),
                FA_LDS_K(fa_crown_phase_kernel<64>));
