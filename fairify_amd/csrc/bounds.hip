// Fused multi-layer bound propagation (IBP and forward-symbolic) on f32 MFMA.  gfx950.
//
// Replaces the reference's per-neuron Python triple loop `neuron_bounds`
// (utils/prune.py:105-164) and its per-neuron Z3 "singular verification" (:276-364) with one
// kernel over thousands of boxes; it is also the bounding primitive of the branch-and-bound
// prover.  Algorithm and error accounting: ops/reference.py:bounds (same arithmetic).
//
// A workgroup (4 wave64) owns G box-rows.  Per row, two blocks (upper U / lower L) of rows are
// kept in LDS, each [rb rows][width]:
//   symbolic: n0 coefficient rows, constant row, error row, interval row, interval-error row
//   ibp     : interval row, interval-error row
// A layer is ONE GEMM   out_U = [U | L] . [W+ ; W-],   out_L = [L | U] . [W+ ; W-]
// of (G*2*rb) x (2*n_in) by (2*n_in) x n_out on v_mfma_f32_16x16x4_f32 with the layer's W staged
// in LDS (W+/W- formed on the fly; error rows negated in the second half so they accumulate
// |W-|).  The epilogue (one thread per (row, neuron)) intersects the symbolic and interval
// bounds, applies the ReLU relaxation to the forms in place, re-seeds the interval rows with
// max(0, bound) and writes the error rows for the next layer.  Only the logit forms (and, on
// request, per-neuron bounds / dead flags) go back to HBM.
#include <stdlib.h>

#include "args.h"

__global__ void __launch_bounds__(FA_THREADS)
fa_bounds_kernel(NetDesc net, BoundArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int n0 = net.dims[0];
  const int G = a.G;
  const bool sym = a.symbolic != 0;
  const int crow = n0;                          // constant row (symbolic)
  const int erow = n0 + 1;                      // form error row (symbolic)
  const int irow = sym ? n0 + 2 : 0;            // interval row
  const int ierow = irow + 1;                   // interval error row
  const int rb = irow + 2;
  const int S = a.stride;
  float* s_lo = smem;                           // [G][n0]
  float* s_hi = s_lo + G * n0;
  float* s_m = s_hi + G * n0;
  float* s_W = s_m + G * n0;                    // [n_in][wstride]
  float* bufA = s_W + a.wfloats;
  float* bufB = bufA + G * 2 * rb * S;
  const int row0 = blockIdx.x * G;
  const int tid = threadIdx.x;
  const float unit = net.unit;

  // ---- stage boxes
  for (int i = tid; i < G * n0; i += FA_THREADS) {
    int g = i / n0, d = i % n0;
    int r = row0 + g;
    float l = 0.f, h = 0.f;
    if (r < a.R) {
      if (a.V > 0) {  // node-row expansion: PA dims take the row's assignment
        const int node = r / a.V, v = r - node * a.V;
        l = a.lo[(size_t)node * n0 + d];
        h = a.hi[(size_t)node * n0 + d];
        for (int k = 0; k < a.npa; ++k)
          if (a.pa_idx[k] == d) l = h = a.values[v * a.npa + k];
      } else {
        l = a.lo[(size_t)r * n0 + d];
        h = a.hi[(size_t)r * n0 + d];
      }
    }
    s_lo[i] = l; s_hi[i] = h; s_m[i] = fmaxf(fabsf(l), fabsf(h));
  }
  __syncthreads();
  // ---- layer-0 inputs: identity forms + [hi | lo] interval rows
  {
    const float g0 = net.g_gemm[0];
    for (int i = tid; i < G * 2 * rb * n0; i += FA_THREADS) {
      const int j = i % n0;
      const int rr = (i / n0) % rb;
      const int o = (i / (n0 * rb)) % 2;
      const int g = i / (n0 * rb * 2);
      const float c = o == 0 ? s_hi[g * n0 + j] : s_lo[g * n0 + j];
      float v;
      if (rr == irow) v = c;
      else if (rr == ierow) v = g0 * fabsf(c);
      else if (rr < n0) v = (rr == j) ? 1.f : 0.f;
      else if (rr == crow) v = 0.f;
      else v = g0 * s_m[g * n0 + j];           // erow
      bufA[((g * 2 + o) * rb + rr) * S + j] = v;
    }
  }
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int M = G * 2 * rb;
  for (int l = 0; l < net.n_layers; ++l) {
    const int n_in = net.dims[l];
    const int n_out = net.dims[l + 1];
    const float* W = a.flat + net.w_off[l];
    const float* bias = a.flat + net.b_off[l];
    const int ws = a.wstride;
    for (int i = tid; i < n_in * n_out; i += FA_THREADS) {
      const int k = i / n_out, j = i % n_out;
      s_W[k * ws + j] = W[i];
    }
    __syncthreads();
    // ---------------- GEMM on MFMA
    const int mtiles = (M + 15) >> 4;
    const int ntiles = (n_out + 15) >> 4;
    for (int t = wave; t < mtiles * ntiles; t += 4) {
      const int mt = t / ntiles, nt = t % ntiles;
      const int m = mt * 16 + (lane & 15);
      const int kq = lane >> 4;
      const bool mval = m < M;
      const int g = m / (2 * rb);
      const int rem = m - g * 2 * rb;
      const int o = rem / rb;
      const int r = rem - o * rb;
      const float* a_own = bufA + ((g * 2 + o) * rb + r) * S;
      const float* a_oth = bufA + ((g * 2 + (1 - o)) * rb + r) * S;
      const float sgn = (r == ierow || (sym && r == erow)) ? -1.f : 1.f;
      const int j = nt * 16 + (lane & 15);
      const bool jval = j < n_out;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int k0 = 0; k0 < n_in; k0 += 4) {
        const int k = k0 + kq;
        const bool kv = k < n_in;
        const float av = (mval && kv) ? a_own[k] : 0.f;
        const float wv = (jval && kv) ? s_W[k * ws + j] : 0.f;
        acc = fa_mfma4(av, fmaxf(wv, 0.f), acc);
      }
      for (int k0 = 0; k0 < n_in; k0 += 4) {
        const int k = k0 + kq;
        const bool kv = k < n_in;
        const float av = (mval && kv) ? sgn * a_oth[k] : 0.f;
        const float wv = (jval && kv) ? s_W[k * ws + j] : 0.f;
        acc = fa_mfma4(av, fminf(wv, 0.f), acc);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int mr = mt * 16 + (lane >> 4) * 4 + i;
        if (mr < M && jval) {
          const int gg = mr / (2 * rb);
          const int rm = mr - gg * 2 * rb;
          const int oo = rm / rb;
          const int rr = rm - oo * rb;
          bufB[((gg * 2 + oo) * rb + rr) * S + j] = acc[i];
        }
      }
    }
    __syncthreads();
    // ---------------- epilogue: intersect, relax, re-seed interval rows, next error rows
    const bool last = (l == net.n_layers - 1);
    const float gg_ = net.g_gemm[l];
    const float gc = net.g_conc;
    const float gi = net.g_one;
    const float gnext = last ? 0.f : net.g_gemm[l + 1];
    const int noff = net.neuron_off[l];
    for (int it = tid; it < G * n_out; it += FA_THREADS) {
      const int g = it / n_out, j = it % n_out;
      const int rglob = row0 + g;
      const bool rv = rglob < a.R;
      float* cu = bufB + ((g * 2 + 0) * rb) * S + j;
      float* cl = bufB + ((g * 2 + 1) * rb) * S + j;
      const float b = bias[j];
      // interval rows
      const float hI = cu[irow * S] + b, lI = cl[irow * S] + b;
      const float eIh = cu[ierow * S] * (1.f + 2.f * gg_) + gg_ * fabsf(b);
      const float eIl = cl[ierow * S] * (1.f + 2.f * gg_) + gg_ * fabsf(b);
      float ub = hI + gi * fabsf(hI) + eIh;
      float lb = lI - gi * fabsf(lI) - eIl;
      // symbolic forms
      float cU = 0.f, cL = 0.f, mnU = 0.f, mxU = 0.f, mgU = 0.f, mnL = 0.f, mxL = 0.f, mgL = 0.f;
      float eU = 0.f, eL = 0.f;
      if (sym) {
        const float* glo = s_lo + g * n0;
        const float* ghi = s_hi + g * n0;
        const float* gm = s_m + g * n0;
        cU = cu[crow * S] + b;
        cL = cl[crow * S] + b;
        mnU = cU; mxU = cU; mgU = fabsf(cU);
        mnL = cL; mxL = cL; mgL = fabsf(cL);
        for (int i = 0; i < n0; ++i) {
          const float u = cu[i * S], v = cl[i * S];
          const float ul = u * glo[i], uh = u * ghi[i];
          const float vl = v * glo[i], vh = v * ghi[i];
          mnU += fminf(ul, uh); mxU += fmaxf(ul, uh); mgU += fabsf(u) * gm[i];
          mnL += fminf(vl, vh); mxL += fmaxf(vl, vh); mgL += fabsf(v) * gm[i];
        }
        eU = cu[erow * S] * (1.f + 2.f * gg_) + gg_ * fabsf(b);
        eL = cl[erow * S] * (1.f + 2.f * gg_) + gg_ * fabsf(b);
        ub = fminf(ub, mxU + gc * mgU + eU);
        lb = fmaxf(lb, mnL - gc * mgL - eL);
      }
      if (rv && a.layer_lb) {
        a.layer_lb[(size_t)rglob * net.n_neurons + noff + j] = lb;
        a.layer_ub[(size_t)rglob * net.n_neurons + noff + j] = ub;
      }
      if (last) {
        if (rv) {
          a.out_lb[rglob] = lb;
          a.out_ub[rglob] = ub;
          if (sym) {
            for (int i = 0; i < n0; ++i) {
              a.Lc[(size_t)rglob * n0 + i] = cl[i * S];
              a.Uc[(size_t)rglob * n0 + i] = cu[i * S];
            }
            a.L0[rglob] = cL; a.Le[rglob] = eL;
            a.U0[rglob] = cU; a.Ue[rglob] = eU;
          }
        }
        continue;
      }
      bool forced = false;
      if (a.dead_in && rv) forced = a.dead_in[(size_t)rglob * net.n_hidden + noff + j] != 0;
      else if (a.dead_part && rv) {
        int node = a.V > 0 ? rglob / a.V : rglob;
        if (a.part_mod) node %= a.part_mod;
        forced = a.dead_part[(size_t)a.node_part[node] * net.n_hidden + noff + j] != 0;
      }
      bool fact = false;
      if (a.phase_in && rv) {   // ReLU-phase rows (symbolic.hip: same rule)
        const int8_t ph = a.phase_in[(size_t)rglob * net.n_hidden + noff + j];
        forced = forced || ph < 0;
        fact = ph > 0;
        if (a.infeas && ((ph < 0 && lb > 0.f) || (ph > 0 && ub < 0.f))) a.infeas[rglob] = 1;
      }
      const bool isdead = ub <= 0.f;
      const bool isact = lb >= 0.f;
      if (rv && a.dead_out) a.dead_out[(size_t)rglob * net.n_hidden + noff + j] = isdead ? 1 : 0;
      const bool zero = isdead || forced;
      const float ih = zero ? 0.f : fmaxf(ub, 0.f);
      const float il = zero ? 0.f : fmaxf(lb, 0.f);
      cu[irow * S] = ih;
      cl[irow * S] = il;
      cu[ierow * S] = gnext * ih;
      cl[ierow * S] = gnext * il;
      if (!sym) continue;
      const float* gm = s_m + g * n0;
      // upper relaxation: identity (stable active, or the upper form T = U + eU >= 0 on the
      // whole box: relu(z) <= T there) / zero / chord over [aa, bb] of T
      float eUn = 0.f, mgUn = 0.f;
      const float aa = mnU - gc * mgU + eU;
      if (zero) {
        for (int i = 0; i <= crow; ++i) cu[i * S] = 0.f;
      } else if (isact || fact || aa >= 0.f) {
        cu[crow * S] = cU;
        eUn = eU;
        mgUn = mgU;
      } else {
        const float bb = mxU + gc * mgU + eU;
        const float s = (bb / (bb - aa)) * (1.f + 4.f * unit);
        const float shift = eU - aa;
        for (int i = 0; i < n0; ++i) {
          const float v = cu[i * S] * s;
          cu[i * S] = v;
          mgUn += fabsf(v) * gm[i];
        }
        const float c = cU * s + s * shift;
        cu[crow * S] = c;
        mgUn += fabsf(c);
        eUn = 4.f * unit * s * (mgU + fabsf(shift));
      }
      // lower relaxation: lambda in {0,1} applied to L(x) - eL
      const float aL = mnL - gc * mgL - eL;
      const float bL = mxL + gc * mgL - eL;
      const bool lam1 = !zero && (isact || ((bL > 0.f) && (bL > -aL)));
      float eLn = 0.f, mgLn = 0.f;
      if (lam1) {
        cl[crow * S] = cL;
        eLn = eL;
        mgLn = mgL;
      } else {
        for (int i = 0; i <= crow; ++i) cl[i * S] = 0.f;
      }
      cu[erow * S] = eUn + gnext * mgUn;
      cl[erow * S] = eLn + gnext * mgLn;
    }
    __syncthreads();
    float* tmp = bufA; bufA = bufB; bufB = tmp;
  }
}

extern "C" size_t fa_bounds_smem(const NetDesc& net, int symbolic, int G, int* stride, int* wstride,
                                 int* wfloats) {
  const int n0 = net.dims[0];
  const int rb = symbolic ? n0 + 4 : 2;
  const int S = net.max_width | 1;            // odd stride: conflict-free column reads
  int ws = 1;
  for (int l = 0; l < net.n_layers; ++l) ws = ws > net.dims[l + 1] ? ws : net.dims[l + 1];
  ws |= 1;
  int wsz = 0;
  for (int l = 0; l < net.n_layers; ++l) wsz = wsz > net.dims[l] * ws ? wsz : net.dims[l] * ws;
  wsz = (wsz + 3) & ~3;
  *stride = S;
  *wstride = ws;
  *wfloats = wsz;
  size_t floats = 3 * (size_t)G * n0 + (size_t)wsz + 2 * (size_t)G * 2 * rb * S;
  floats = (floats + 3) & ~(size_t)3;
  return floats * sizeof(float);
}

extern "C" int fa_sym_try_launch(const NetDesc& net, BoundArgs a, unsigned long long fold_mask,
                                 hipStream_t stream);

static int fa_lds_only() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("FAIRIFY_BOUNDS_KERNEL");
    v = (e && e[0] == 'l') ? 1 : 0;   // "lds": force the LDS-tiled kernel (A/B comparisons)
  }
  return v;
}

extern "C" int fa_bounds_launch(const NetDesc& net, BoundArgs args, hipStream_t stream) {
  if (args.R <= 0) return 0;
  if (args.symbolic && !fa_lds_only()) {
    unsigned long long fold = args.fold;
    if (args.V > 0)
      for (int k = 0; k < args.npa; ++k) fold |= 1ull << args.pa_idx[k];
    const int rc = fa_sym_try_launch(net, args, fold, stream);
    if (rc == 1) return 0;
    if (rc < 0) return -rc;
  }
  const size_t limit = 160 * 1024;
  int G = args.G > 0 ? args.G : 16;
  int S = 0, ws = 0, wf = 0;
  size_t bytes = 0;
  for (;;) {
    bytes = fa_bounds_smem(net, args.symbolic, G, &S, &ws, &wf);
    if (bytes <= 64 * 1024 || G == 1) break;
    G--;
  }
  if (bytes > limit) return -1;
  args.G = G;
  args.stride = S;
  args.wstride = ws;
  args.wfloats = wf;
  if (!fa_lds_ok(bytes)) return -4;       // fa_lds_prepare() not run (Backend construction)
  dim3 grid((args.R + G - 1) / G);
  hipLaunchKernelGGL(fa_bounds_kernel, grid, dim3(FA_THREADS), bytes, stream, net, args);
  return (int)hipGetLastError();
}

FA_LDS_REGISTER(FA_LDS_K(fa_bounds_kernel));
