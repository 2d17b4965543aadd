// Branch-and-bound node test: fairness-pair LP certificate (ops/reference.py:pair_certify).
//
// fa_pair_eval_kernel : one thread per (node, PA pair, orientation) evaluates the convex
//                       piecewise-linear certificate g(t) at t in {0, 1} and at every breakpoint
//                       of the shared-feature coefficients and keeps min_t g(t) and its argmin;
//                       pairs already excluded by the rows' rigorous sign bounds get g = -1.
// fa_pair_fused_kernel: eval + pick in one launch when a node has at most FA_CERT_FUSE_Q
//                       (pair, orientation) entries (the common single-binary-PA case): one lane
//                       per entry, shuffle arg-max per node, the node's first lane picks.
// fa_pair_pick_kernel : one thread per node picks the most violating pair/orientation, and for
//                       it emits the per-dimension split scores (|coef| x width at t*), the best
//                       split dimension, the leaf flag and the candidate vertex pair (x, x') that
//                       maximises the objective (PA values set, relaxed features clipped to tau).
#include "args.h"

// Folded form of one row: coefficient i (0 on PA dims), constant (incl. err sign and PA terms),
// |PA contribution| for the rounding margin.
struct Form {
  const float* c;
  float c0;
  float fmag;
};

__device__ __forceinline__ bool fa_is_pa(const CertArgs& a, int d) {
  for (int k = 0; k < a.npa; ++k)
    if (a.pa_idx[k] == d) return true;
  return false;
}

__device__ __forceinline__ Form fa_fold(const CertArgs& a, const float* C, float c0, int v) {
  Form f;
  f.c = C;
  float contrib = 0.f, cmag = 0.f;
  for (int k = 0; k < a.npa; ++k) {
    const float t = C[a.pa_idx[k]] * (float)a.values[v * a.npa + k];
    contrib += t;
    cmag += fabsf(t);          // the products' magnitudes: with several PA dims the sum can cancel
  }
  f.c0 = c0 + contrib;
  f.fmag = cmag;
  return f;
}

// A / B forms of pair q (orientation o) of node n, with sign applied through sA / sB.
__device__ __forceinline__ void fa_pair_forms(const CertArgs& a, int n, int q, int o, Form& A, float& sA,
                                              Form& B, float& sB) {
  const int vi = (int)a.pairs[2 * q], vj = (int)a.pairs[2 * q + 1];
  const size_t ri = (size_t)n * a.V + vi, rj = (size_t)n * a.V + vj;
  if (o == 0) {  // t * (-(L_v(x) - eL)) + (1-t) * (U_v'(x') + eU)
    A = fa_fold(a, a.Lc + ri * a.n0, a.L0[ri] - a.Le[ri], vi);
    sA = -1.f;
    B = fa_fold(a, a.Ucp + rj * a.n0, a.U0p[rj] + a.Uep[rj], vj);
    sB = 1.f;
  } else {       // t * (U_v(x) + eU) + (1-t) * (-(L_v'(x') - eL))
    A = fa_fold(a, a.Uc + ri * a.n0, a.U0[ri] + a.Ue[ri], vi);
    sA = 1.f;
    B = fa_fold(a, a.Lcp + rj * a.n0, a.L0p[rj] - a.Lep[rj], vj);
    sB = -1.f;
  }
}

__device__ float fa_g_at(const CertArgs& a, int n, const Form& A, float sA, const Form& B, float sB, float t,
                         float magA, float magB) {
  const float* xl = a.xlo + (size_t)n * a.n0;
  const float* xh = a.xhi + (size_t)n * a.n0;
  const float* pl = a.xplo + (size_t)n * a.n0;
  const float* ph = a.xphi + (size_t)n * a.n0;
  float val = 0.f;
  for (int i = 0; i < a.n0; ++i) {
    if (fa_is_pa(a, i)) continue;
    const float ai = sA * A.c[i];
    const float bi = sB * B.c[i];
    if (a.shared[i]) {
      const float cs = t * ai + (1.f - t) * bi;
      val += fmaxf(cs * xl[i], cs * xh[i]);
    } else {
      const float ca = t * ai, cb = (1.f - t) * bi;
      val += fmaxf(ca * xl[i], ca * xh[i]) + fmaxf(cb * pl[i], cb * ph[i]);
    }
  }
  const float A0 = sA * A.c0, B0 = sB * B.c0;
  float g = val + t * A0 + (1.f - t) * B0;
  g += a.gmarg * (t * magA + (1.f - t) * magB) + 8.f * a.unit * (magA + magB);
  return g;
}

__device__ void fa_mags(const CertArgs& a, int n, const Form& A, const Form& B, float& magA, float& magB) {
  const float* xl = a.xlo + (size_t)n * a.n0;
  const float* xh = a.xhi + (size_t)n * a.n0;
  const float* pl = a.xplo + (size_t)n * a.n0;
  const float* ph = a.xphi + (size_t)n * a.n0;
  magA = fabsf(A.c0) + A.fmag;
  magB = fabsf(B.c0) + B.fmag;
  for (int i = 0; i < a.n0; ++i) {
    if (fa_is_pa(a, i)) continue;
    magA += fabsf(A.c[i]) * fmaxf(fabsf(xl[i]), fabsf(xh[i]));
    magB += fabsf(B.c[i]) * fmaxf(fabsf(pl[i]), fabsf(ph[i]));
  }
}

// Register-resident evaluation: the pair's two folded forms and the node boxes are loaded once
// (NM >= n0, compile-time), then g(t) is evaluated at t in {0, 1} and at every breakpoint of a
// shared feature without touching memory again.  Same arithmetic as fa_g_at / fa_mags.
#define FA_CERT_THREADS 64
// min_t g(t) of pair qq (orientation-major) of node n -> (gmin, tstar)
template <int NM>
__device__ __forceinline__ void fa_pair_eval_one(const CertArgs& a, int n, int qq, float& gmin, float& tstar) {
  const int o = qq / a.Pp, q = qq % a.Pp;
  const int vi = (int)a.pairs[2 * q], vj = (int)a.pairs[2 * q + 1];
  {  // exact-sign shortcut from the rigorous per-row bounds
    const size_t ri = (size_t)n * a.V + vi, rj = (size_t)n * a.V + vj;
    const bool imp = (o == 0) ? (a.olb[ri] >= 0.f || a.oubp[rj] <= 0.f) : (a.oub[ri] <= 0.f || a.olbp[rj] >= 0.f);
    if (imp) {
      gmin = -1.f;
      tstar = 0.f;
      return;
    }
  }
  Form A, B;
  float sA, sB;
  fa_pair_forms(a, n, q, o, A, sA, B, sB);
  const int n0 = a.n0;
  const float* xlp = a.xlo + (size_t)n * n0;
  const float* xhp = a.xhi + (size_t)n * n0;
  const float* plp = a.xplo + (size_t)n * n0;
  const float* php = a.xphi + (size_t)n * n0;
  float ca[NM], cb[NM], xl[NM], xh[NM], pl[NM], ph[NM];
  bool sh[NM], un[NM];
  float magA = fabsf(A.c0) + A.fmag, magB = fabsf(B.c0) + B.fmag;
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    const bool v = i < n0 && !fa_is_pa(a, i);
    ca[i] = v ? sA * A.c[i] : 0.f;
    cb[i] = v ? sB * B.c[i] : 0.f;
    xl[i] = v ? xlp[i] : 0.f;
    xh[i] = v ? xhp[i] : 0.f;
    pl[i] = v ? plp[i] : 0.f;
    ph[i] = v ? php[i] : 0.f;
    sh[i] = v && a.shared[i];
    un[i] = v && !a.shared[i];
    magA += fabsf(ca[i]) * fmaxf(fabsf(xl[i]), fabsf(xh[i]));
    magB += fabsf(cb[i]) * fmaxf(fabsf(pl[i]), fabsf(ph[i]));
  }
  const float A0 = sA * A.c0, B0 = sB * B.c0;
  const float marg0 = 8.f * a.unit * (magA + magB);
  auto g_at = [&](float t) __attribute__((always_inline)) {
    float val = 0.f;
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      const float cs = t * ca[i] + (1.f - t) * cb[i];
      const float c1 = t * ca[i], c2 = (1.f - t) * cb[i];
      const float vs = fmaxf(cs * xl[i], cs * xh[i]);
      const float vu = fmaxf(c1 * xl[i], c1 * xh[i]) + fmaxf(c2 * pl[i], c2 * ph[i]);
      val += sh[i] ? vs : (un[i] ? vu : 0.f);
    }
    return val + t * A0 + (1.f - t) * B0 + a.gmarg * (t * magA + (1.f - t) * magB) + marg0;
  };
  float best = g_at(0.f), bt = 0.f;
  {
    const float g1 = g_at(1.f);
    if (g1 < best) { best = g1; bt = 1.f; }
  }
  if constexpr (NM <= 16) {
    // unrolled over the register arrays (no select chain per breakpoint); same breakpoints in the
    // same order as the runtime loop below, so bitwise the same (gmin, t*)
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      if (!sh[i]) continue;                 // uniform: shared flag of dim i (false beyond n0)
      const float den = ca[i] - cb[i];
      if (den == 0.f) continue;
      const float t = -cb[i] / den;
      if (!(t > 0.f && t < 1.f)) continue;
      const float g = g_at(t);
      if (g < best) { best = g; bt = t; }
    }
  } else {
#pragma unroll 1
    for (int i = 0; i < n0; ++i) {
      // runtime loop over breakpoints; the register arrays are read through a select chain
      float ai = 0.f, bi = 0.f;
      bool s_i = false;
#pragma unroll
      for (int k = 0; k < NM; ++k)
        if (k == i) { ai = ca[k]; bi = cb[k]; s_i = sh[k]; }
      if (!s_i) continue;
      const float den = ai - bi;
      if (den == 0.f) continue;
      const float t = -bi / den;
      if (!(t > 0.f && t < 1.f)) continue;
      const float g = g_at(t);
      if (g < best) { best = g; bt = t; }
    }
  }
  gmin = best;
  tstar = bt;
}

template <int NM>
__global__ void __launch_bounds__(FA_CERT_THREADS) fa_pair_eval_kernel(CertArgs a) {
  const int Q = a.Pp * a.norient;
  const int64_t idx = (int64_t)blockIdx.x * FA_CERT_THREADS + threadIdx.x;
  if (idx >= (int64_t)a.Nn * Q) return;
  float g = -INFINITY, t = 0.f;
  const int n = (int)(idx / Q);
  const int8_t st = a.status ? a.status[a.part[n]] : (int8_t)3;
  if (st == 3 || st == 4) fa_pair_eval_one<NM>(a, n, (int)(idx % Q), g, t);
  a.gmin[idx] = g;
  a.tstar[idx] = t;
}

// most violating pair (bq, its g = bg, its t*) of node n -> open flag, split scores, candidate
template <int NM>
__device__ __forceinline__ void fa_pick_node(const CertArgs& a, int n, float bg, int bq, float t);

template <int NM>
__global__ void __launch_bounds__(FA_CERT_THREADS) fa_pair_pick_kernel(CertArgs a) {
  const int n = blockIdx.x * FA_CERT_THREADS + threadIdx.x;
  if (n >= a.Nn) return;
  const int Q = a.Pp * a.norient;
  float bg = -INFINITY;
  int bq = 0;
  for (int qq = 0; qq < Q; ++qq) {
    float g = a.gmin[(size_t)n * Q + qq];
    if (g != g) g = INFINITY;     // a non-finite certificate value never closes a node
    if (g > bg) { bg = g; bq = qq; }
  }
  fa_pick_node<NM>(a, n, bg, bq, a.tstar[(size_t)n * Q + bq]);
}

// Eval + pick fused for nodes with at most FA_CERT_FUSE_Q (pair, orientation) entries: a group
// of QG = next_pow2(Q) consecutive lanes per node evaluates one entry each, a shuffle arg-max
// inside the group keeps the first maximum (the two-kernel path's rule), and the group's first
// lane runs the pick.  One launch instead of two per BaB sub-batch, no gmin / tstar round trip.
#ifndef FA_CERT_WPE16
#define FA_CERT_WPE16 1
#endif
template <int NM>
__global__ void __launch_bounds__(FA_CERT_THREADS) __attribute__((amdgpu_waves_per_eu(NM == 16 ? FA_CERT_WPE16 : 1)))
fa_pair_fused_kernel(CertArgs a, int QG) {
  const int Q = a.Pp * a.norient;
  const int gidx = blockIdx.x * FA_CERT_THREADS + threadIdx.x;
  const int n = gidx / QG, qq = gidx - n * QG;
  bool live = n < a.Nn && qq < Q;
  if (live && a.status) {   // node of a decided / stopped partition: closed, nothing evaluated
    const int8_t st = a.status[a.part[n]];
    live = st == 3 || st == 4;
  }
  float g = -INFINITY, t = 0.f;
  if (live) fa_pair_eval_one<NM>(a, n, qq, g, t);
  if (g != g) g = INFINITY;       // NaN -> keep the node open (same rule as fa_pair_pick_kernel)
  int bq = live ? qq : 0x7fffffff;
  for (int o = 1; o < QG; o <<= 1) {     // groups are aligned to QG lanes (QG divides 64)
    const float g2 = __shfl_xor(g, o);
    const float t2 = __shfl_xor(t, o);
    const int q2 = __shfl_xor(bq, o);
    if (g2 > g || (g2 == g && q2 < bq)) { g = g2; t = t2; bq = q2; }
  }
  if (n < a.Nn && qq == 0) fa_pick_node<NM>(a, n, g, bq == 0x7fffffff ? 0 : bq, t);
}

// Register-resident pick (NM >= n0, compile-time): the pair's coefficients and the node's boxes
// are loaded once with independent loads, every per-dimension loop is unrolled.  A node's pick is
// one lane's serial work, so at a small BFS level (a 1/8 shard) its memory round trips ARE the
// kernel's duration: the per-dimension loads of the old runtime loops and the smear's one
// neuron-at-a-time loads cost ~100 us per launch (profiles/r4/emu/).
template <int NM>
__device__ __forceinline__ void fa_pick_node(const CertArgs& a, int n, float bg, int bq, float t) {
  if (a.skip_closed && !(bg > 0.f)) {
    a.open[n] = 0;
    a.score[n] = bg;
    if (a.leaf) a.leaf[n] = 0;
    return;
  }
  const int o = bq / a.Pp, q = bq % a.Pp;
  Form A, B;
  float sA, sB;
  fa_pair_forms(a, n, q, o, A, sA, B, sB);
  const int n0 = a.n0;
  const float* xlp = a.xlo + (size_t)n * n0;
  const float* xhp = a.xhi + (size_t)n * n0;
  const float* plp = a.xplo + (size_t)n * n0;
  const float* php = a.xphi + (size_t)n * n0;
  float* cxo = a.cand_x + (size_t)n * n0;
  float* cpo = a.cand_xp + (size_t)n * n0;
  float* sco = a.scores ? a.scores + (size_t)n * 2 * n0 : nullptr;
  float ai[NM], bi[NM], xl[NM], xh[NM], pl[NM], ph[NM];
  unsigned pam = 0u, shm = 0u;   // protected / shared dims (bit masks: bool arrays stay in scratch)
  for (int k = 0; k < a.npa; ++k) pam |= 1u << a.pa_idx[k];
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    const bool v = i < n0;
    if (v && a.shared[i]) shm |= 1u << i;
    const bool p = (pam >> i) & 1u;
    ai[i] = (v && !p) ? sA * A.c[i] : 0.f;
    bi[i] = (v && !p) ? sB * B.c[i] : 0.f;
    xl[i] = v ? xlp[i] : 0.f;
    xh[i] = v ? xhp[i] : 0.f;
    pl[i] = v ? plp[i] : 0.f;
    ph[i] = v ? php[i] : 0.f;
  }
  float bs = -1.f;
  int bd = 0;
  bool leaf = true;
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    if (i >= n0) continue;
    const float wx = xh[i] - xl[i];
    const float cs = t * ai[i] + (1.f - t) * bi[i];
    float sx, cx;
    if (((shm >> i) & 1u)) {
      sx = fabsf(cs) * wx;
      cx = cs > 0.f ? xh[i] : xl[i];
    } else {
      sx = fabsf(t * ai[i]) * wx;
      cx = (t * ai[i] > 0.f) ? xh[i] : xl[i];
    }
    sx += 1e-9f * wx;
    if (((pam >> i) & 1u) || wx <= 0.f) sx = -1.f;
    if (!((pam >> i) & 1u) && wx > 0.f) leaf = false;
    if (sx > bs) { bs = sx; bd = i; }
    if (sco) sco[i] = sx;
    cxo[i] = cx;
    cpo[i] = ((shm >> i) & 1u) ? cx : (((1.f - t) * bi[i] > 0.f) ? ph[i] : pl[i]);
  }
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    if (i >= n0) continue;
    float sxp = -1.f;
    if (!((shm >> i) & 1u) && !((pam >> i) & 1u)) {
      const float wxp = ph[i] - pl[i];
      if (wxp > 0.f) {
        sxp = fabsf((1.f - t) * bi[i]) * wxp + 1e-9f * wxp;
        leaf = false;
      }
    }
    if (sco) sco[n0 + i] = sxp;
    if (sxp > bs) { bs = sxp; bd = n0 + i; }
  }
  if (a.smear && sco && a.nra == 0 && n0 <= NM) {
    // first-layer smear: sum over the node's rows of |W0[i, j]| over layer-0 neurons j that are
    // unstable on the row's box, times the width of dim i.  The unstable set comes 32 neurons at a
    // time from independent loads into a bit mask; the |W0| rows (transposed, NM wide) of two
    // unstable neurons are fetched together; accumulation in ascending j as before.
    float acc[NM];
#pragma unroll
    for (int i = 0; i < NM; ++i) acc[i] = 0.f;
    for (int v = 0; v < a.V; ++v) {
      const float* lb = a.lay_lb + ((size_t)n * a.V + v) * a.lay_N;
      const float* ub = a.lay_ub + ((size_t)n * a.V + v) * a.lay_N;
      for (int j0 = 0; j0 < a.n1; j0 += 32) {
        unsigned msk = 0u;
#pragma unroll
        for (int k = 0; k < 32; ++k) {
          const int j = j0 + k;
          const bool jv = j < a.n1;
          const float l = jv ? lb[j] : 0.f, u = jv ? ub[j] : 0.f;
          if (l < 0.f && u > 0.f) msk |= 1u << k;
        }
        while (msk) {
          int jj[2];
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            jj[k] = msk ? j0 + __builtin_ctz(msk) : -1;
            msk &= msk - 1u;
          }
          float4 w[2][NM / 4];
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const float4* wr = reinterpret_cast<const float4*>(a.W0T + (size_t)(jj[k] < 0 ? 0 : jj[k]) * NM);
#pragma unroll
            for (int i4 = 0; i4 < NM / 4; ++i4) w[k][i4] = wr[i4];
          }
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            if (jj[k] < 0) break;
#pragma unroll
            for (int i4 = 0; i4 < NM / 4; ++i4) {
              acc[4 * i4] += w[k][i4].x;
              acc[4 * i4 + 1] += w[k][i4].y;
              acc[4 * i4 + 2] += w[k][i4].z;
              acc[4 * i4 + 3] += w[k][i4].w;
            }
          }
        }
      }
    }
    bs = -1.f;
    bd = 0;
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      if (i >= n0) continue;
      const float wx = xh[i] - xl[i];
      float sx = acc[i] * wx + 1e-9f * wx;
      if (((pam >> i) & 1u) || wx <= 0.f) sx = -1.f;
      sco[i] = sx;
      if (sx > bs) { bs = sx; bd = i; }
    }
  }
  // candidate pair: PA values of the chosen pair, relaxed features within tau of x (and in x' box)
  const int vi = (int)a.pairs[2 * q], vj = (int)a.pairs[2 * q + 1];
  for (int k = 0; k < a.npa; ++k) {
    cxo[a.pa_idx[k]] = (float)a.values[vi * a.npa + k];
    cpo[a.pa_idx[k]] = (float)a.values[vj * a.npa + k];
  }
  for (int k = 0; k < a.nra; ++k) {
    const int r = a.ra_idx[k];
    const float v = fminf(fmaxf(cpo[r], cxo[r] - a.tau), cxo[r] + a.tau);
    cpo[r] = fminf(fmaxf(v, plp[r]), php[r]);
  }
  a.open[n] = bg > 0.f ? 1 : 0;
  a.score[n] = bg;
  a.split_dim[n] = bd;
  a.cand_v[n] = q;
  a.cand_o[n] = o;
  if (a.leaf) a.leaf[n] = leaf ? 1 : 0;
}

// pairs x orientations up to which eval and pick run fused (one thread per node); more pairs
// keep one thread per (node, pair) so wide PA tables still fill the chip
#ifndef FA_CERT_FUSE_Q
#define FA_CERT_FUSE_Q 4
#endif

extern "C" int fa_certify_launch(CertArgs a, hipStream_t stream) {
  if (a.Nn <= 0) return 0;
  if (a.npa > FA_CMAX_PA || a.nra > FA_MAX_RA) return -3;
  const int64_t tot = (int64_t)a.Nn * a.Pp * a.norient;
  if (a.Pp * a.norient <= FA_CERT_FUSE_Q && a.n0 <= 32) {
    int QG = 1;
    while (QG < a.Pp * a.norient) QG <<= 1;
    const dim3 gn((unsigned)(((int64_t)a.Nn * QG + FA_CERT_THREADS - 1) / FA_CERT_THREADS));
    if (a.n0 <= 16) hipLaunchKernelGGL(fa_pair_fused_kernel<16>, gn, dim3(FA_CERT_THREADS), 0, stream, a, QG);
    else hipLaunchKernelGGL(fa_pair_fused_kernel<32>, gn, dim3(FA_CERT_THREADS), 0, stream, a, QG);
    return (int)hipGetLastError();
  }
  const dim3 ge((unsigned)((tot + FA_CERT_THREADS - 1) / FA_CERT_THREADS));
  if (a.n0 <= 16) hipLaunchKernelGGL(fa_pair_eval_kernel<16>, ge, dim3(FA_CERT_THREADS), 0, stream, a);
  else if (a.n0 <= 32) hipLaunchKernelGGL(fa_pair_eval_kernel<32>, ge, dim3(FA_CERT_THREADS), 0, stream, a);
  else return -4;
  const dim3 gp((a.Nn + FA_CERT_THREADS - 1) / FA_CERT_THREADS);
  if (a.n0 <= 16) hipLaunchKernelGGL(fa_pair_pick_kernel<16>, gp, dim3(FA_CERT_THREADS), 0, stream, a);
  else hipLaunchKernelGGL(fa_pair_pick_kernel<32>, gp, dim3(FA_CERT_THREADS), 0, stream, a);
  return (int)hipGetLastError();
}
