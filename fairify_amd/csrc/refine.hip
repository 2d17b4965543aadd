// Back-substituted hidden-layer bounds (CROWN for intermediate neurons) between the forward
// symbolic pass and the backward output pass of the branch-and-bound (K4 refinement).  gfx950.
// Same arithmetic and error terms as ops/reference.py:crown_refine / _backsub.
//
// Why: the forward pass (symbolic.hip) relaxes each layer with the linear forms it carried
// forward, so on deep networks the per-neuron pre-activation intervals loosen with depth, and every
// later relaxation -- including the output pass of crown.hip -- inherits that slack.  Bounding
// each hidden neuron z_k[j] = W_k[:, j] . h_{k-1} + b_k[j] by back-substitution to the input box
// (through the relaxations of layers k-1 .. 0, their intervals already refined) is what the
// reference's per-partition Z3 check gets for free from exact case splits
// (utils/verif_utils.py:525-528, src/AC/Verify-AC.py:146-158): on the bench's AC-7 (13-64-32-16-8-4)
// residue a partition closes with a median of ~800 BaB nodes instead of > 32 768
// (tools/diag_open_nodes.py --bound fullcrown, profiles/r4/refine/).
//
// Mapping: one workgroup (4 wave64s) owns G box-rows; their per-neuron bounds live in an LDS slab
// for the whole kernel.  Per target layer k the (row, sign, neuron) triples of the G rows are the
// "virtual columns": 16 per MFMA tile, so a multiplier vector lives transposed in registers (reg i
// of tile t = neuron 16t + 4 (lane >> 4) + i of column lane & 15) and lambda' = W_l mu runs as a
// v_mfma_f32_16x16x4_f32 chain with W_l staged once per workgroup in backward operand order
// (the layout of fa_crown_mfma_kernel), plus the |W| |mu| chain of the rounding term.  Each column
// concretises its form at its row's box and tightens the slab (max of lower, min of upper bounds:
// both are rigorous); a workgroup barrier separates the layers; the slab goes back to global memory
// at the end.  Columns of one tile may belong to different rows (narrow layers pack several rows
// per tile).  Only UNSTABLE neurons get columns (compacted per layer with an LDS counter): a stable
// neuron's relaxation is exact, so its interval only enters rounding terms.  Each neuron's
// relaxation (slopes, offset, rounding magnitude) is computed once per row when its layer is final
// (fa_refine_records), not per column and layer; the rows' boxes are staged in LDS.
#include <hip/hip_runtime.h>

#include <stdlib.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "args.h"

// Mode FULL (fa_backward_launch): no forward pass at all -- layer 0 from the box, every hidden layer
// by back-substitution, then the logit's forms and bounds (the work of crown.hip) in the same
// launch: one kernel instead of forward symbolic + refine + output pass (ops/reference.py:
// backward_bounds).  Mode REFINE (fa_refine_launch): tighten the forward pass's hidden-layer bounds.
struct RefineCfg {
  int w_lds[FA_MAX_LAYERS];   // LDS float offset of layer l's W in backward operand order
  int b_lds[FA_MAX_LAYERS];
  int slab;                   // LDS float offset of the row slabs: G x [lb (N) | ub (N)]
  int rec;                    // G x n_hidden float4 relaxation records (fa_refine_records)
  int hm;                     // G x n_hidden: max(ub, 0) of live neurons (the GEMM rounding terms)
  int box;                    // G x [xl (n0) | xh (n0)], protected attributes fixed
  int list;                   // G x max width ints: the current layer's columns
  int rrun;                   // G running-row flags + the column counter
  int G;                      // box-rows per workgroup
  int floats;
  int full;                   // 1: mode FULL
  int logit;                  // REFINE mode: also the logit's backward forms (the work of crown.hip),
                              // kept where tighter than the forward ones (FULL: always)
};

__device__ __forceinline__ float fa_rgam(int k, float u) {
  const float ku = (float)(k + 2) * u;
  return ku / (1.f - ku) * (1.f + 4.f * u);
}

__device__ __forceinline__ const uint8_t* fa_refine_dmask(const NetDesc& net, const BoundArgs& a, int r) {
  if (a.dead_in) return a.dead_in + (size_t)r * net.n_hidden;
  if (a.dead_part) {
    const int node = a.V > 0 ? r / a.V : r;
    return a.dead_part + (size_t)a.node_part[a.part_mod ? node % a.part_mod : node] * net.n_hidden;
  }
  return nullptr;
}

// the +-1 multiplier of a hidden neuron's relaxation, per (row, neuron) once its bounds are final:
// x = slope for a multiplier >= 0, y = slope for one < 0, z = lb (unstable only: the upper
// relaxation's offset), w = max(|lb|, |ub|) (unstable only: the offset's rounding term).  Stable
// neurons get slopes 1/1 or 0/0 and z = w = 0, so the column loop needs no branches and no
// division (ops/reference.py:_backsub, same values).
__device__ __forceinline__ void fa_refine_records(const NetDesc& net, const BoundArgs& a, const RefineCfg& cfg,
                                                  int l, int rb, float* smem) {
  const int N = net.n_neurons, NH = net.n_hidden;
  const int n = net.dims[l + 1], off = net.neuron_off[l];
  const float u = net.unit;
  const float* slab = smem + cfg.slab;
  float4* rec = reinterpret_cast<float4*>(smem + cfg.rec);
  float* hmx = smem + cfg.hm;
  for (int e = threadIdx.x; e < cfg.G * n; e += blockDim.x) {
    const int g = e / n, jj = e - g * n, h = off + jj;
    const int r = min(rb + g, a.R - 1);
    const int ph = a.phase_in ? (int)a.phase_in[(size_t)r * NH + h] : 0;
    // a fixed phase (ReLU-phase BaB rows) holds on the node's region: fixed active -> exact identity
    // (lb >= 0 there), fixed inactive -> exactly 0
    const float lb = ph > 0 ? fmaxf(slab[g * 2 * N + h], 0.f) : slab[g * 2 * N + h];
    const float ub = ph < 0 ? fminf(slab[g * 2 * N + N + h], 0.f) : slab[g * 2 * N + N + h];
    bool dd = ub <= 0.f || ph < 0;
    const uint8_t* dm = fa_refine_dmask(net, a, r);
    if (dm && dm[h]) dd = true;
    const bool act = !dd && (lb >= 0.f || ph > 0);
    const bool unst = !dd && !act;
    const float alpha = ub > -lb ? 1.f : 0.f;
    const float sl = unst ? (ub / (ub - lb)) * (1.f + 4.f * u) : 0.f;
    float4 q;
    q.x = act ? 1.f : (dd ? 0.f : alpha);
    q.y = act ? 1.f : (dd ? 0.f : sl);
    q.z = unst ? lb : 0.f;
    q.w = unst ? fmaxf(fabsf(lb), fabsf(ub)) : 0.f;
    rec[g * (NH + 1) + h] = q;
    hmx[g * (NH + 1) + h] = dd ? 0.f : fmaxf(ub, 0.f);
  }
}

// One back-substitution step of a column through layer l (its relaxation records, then W_l):
// lam <- W_l (relaxed lam), constant and rounding terms accumulated.  LC >= 0: l is the compile-time
// layer LC of shape S (widths constant, tile loops without trip-count checks).
template <int TM, bool WG, class S, int LC>
__device__ __forceinline__ void fa_refine_step(const NetDesc& net, const RefineCfg& cfg, const float* smem,
                                               const float* wsrc, const float4* recg, const float* hmg,
                                               const float* bl, int n0, int lane, float u, int l_rt,
                                               float (&lam)[TM][4], float& c, float& err) {
  constexpr bool CS = S::L > 0 && LC >= 0;
  const int l = CS ? LC : l_rt;
  auto D = [&](int i) { return CS ? S::dim(i) : net.dims[i]; };
  const int grp = lane >> 4;
  const int n = D(l + 1);
  const int nin = D(l);
  const int tout = (n + 15) >> 4, tin = (nin + 15) >> 4;
  const int off = net.neuron_off[l];
  const float* b = smem + cfg.b_lds[l];
  float mu[TM][4];
  float cs = 0.f, cm = 0.f, er = 0.f;
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    if (t >= tout) break;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int jj = 16 * t + 4 * grp + i;
      const bool jv = jj < n;
      // clamped index + select, not a guarded load (an exec-mask branch: SALU)
      const int jc = min(jj, n - 1);
      const float4 qr = recg[off + jc];
      const float br = b[jc];
      const float4 q = jv ? qr : make_float4(0.f, 0.f, 0.f, 0.f);
      const float bj = jv ? br : 0.f;
      const float lm = lam[t][i];
      const bool neg = lm < 0.f;
      const float m = lm * (neg ? q.y : q.x);
      const float tt = neg ? -m * q.z : 0.f;
      mu[t][i] = m;
      cs += m * bj + tt;
      cm += fabsf(m * bj) + fabsf(tt);
      er += neg ? 3.f * u * (fabsf(m) * q.w + fabsf(tt)) : 0.f;
    }
  }
  const float4* wb = reinterpret_cast<const float4*>(wsrc + cfg.w_lds[l]);
  const float gn = fa_rgam(2 * n + 1, u);
  const int hoff = l > 0 ? net.neuron_off[l - 1] : 0;
#pragma unroll
  for (int ot = 0; ot < TM; ++ot) {
    if (ot >= tin) break;
    f32x4 Z = {0.f, 0.f, 0.f, 0.f}, Q = Z;
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      if (t >= tout) break;
      const float4 w4 = wb[(ot * tout + t) * 64 + lane];
      const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        Z = fa_mfma4(wv[i], mu[t][i], Z);
        Q = fa_mfma4(fabsf(wv[i]), fabsf(mu[t][i]), Q);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int in = 16 * ot + 4 * grp + i;
      const int ic = min(in, nin - 1);
      const float hr = l > 0 ? hmg[hoff + ic] : fmaxf(fabsf(bl[ic]), fabsf(bl[n0 + ic]));
      const float hm = in < nin ? hr : 0.f;
      lam[ot][i] = in < nin ? Z[i] : 0.f;
      er += gn * Q[i] * hm;
    }
  }
#pragma unroll
  for (int ot = 0; ot < TM; ++ot)
    if (ot >= tin)
#pragma unroll
      for (int i = 0; i < 4; ++i) lam[ot][i] = 0.f;
  // per-column sums over the 4 lane groups holding the column's neurons
  cs += __shfl_xor(cs, 16); cs += __shfl_xor(cs, 32);
  cm += __shfl_xor(cm, 16); cm += __shfl_xor(cm, 32);
  er += __shfl_xor(er, 16); er += __shfl_xor(er, 32);
  const float gc = fa_rgam(2 * n + 1, u);
  const float cold = c;
  c = cold + cs;
  err += er + gc * (fabsf(cold) + cm);
}

template <int TM, bool WG, class S, int KC, int... IS>
__device__ __forceinline__ void fa_refine_back_c(std::integer_sequence<int, IS...>, const NetDesc& net,
                                                 const RefineCfg& cfg, const float* smem, const float* wsrc,
                                                 const float4* recg, const float* hmg, const float* bl, int n0,
                                                 int lane, float u, float (&lam)[TM][4], float& c, float& err) {
  // layers KC-1 .. 0 in order, each a compile-time step
  (fa_refine_step<TM, WG, S, KC - 1 - IS>(net, cfg, smem, wsrc, recg, hmg, bl, n0, lane, u, 0, lam, c, err), ...);
}

// One 16-column tile of layer k: the columns' multipliers start at +-W_k[:, j], are carried back to
// the input box (fa_refine_step per layer) and concretised; the slab (and, for the logit, the
// output forms) tightened.  KC >= 0: k is the compile-time layer KC of shape S.
template <int TM, bool WG, class S, int KC>
__device__ __forceinline__ void fa_refine_col(const NetDesc& net, const BoundArgs& a, const RefineCfg& cfg,
                                              const float* smem, const float* wsrc, float* slab,
                                              const float4* rec, const float* hmx, const float* box,
                                              const int* list, int k_rt, int rb, int nv, int tile, int lane,
                                              float gK, float g0, float g1) {
  constexpr bool CS = S::L > 0 && KC >= 0;
  const int k = CS ? KC : k_rt;
  auto D = [&](int i) { return CS ? S::dim(i) : net.dims[i]; };
  const int L = CS ? S::L : net.n_layers;
  const int col = lane & 15, grp = lane >> 4;
  const int n0 = D(0);
  const int N = net.n_neurons, NH = net.n_hidden;
  const float u = net.unit;
  const bool logit = k == L - 1;
  const int nk = D(k + 1);
  const int ktop = D(k);
  const int offk = net.neuron_off[k];
  const int tk = (nk + 15) >> 4;
  const float* wk = wsrc + cfg.w_lds[k];
  const int idx0 = tile * 16 + col;
  const bool vvalid = idx0 < nv;
  const int idx = vvalid ? idx0 : nv - 1;
  const int e = list[idx >> 1];
  const int s = idx & 1;
  const int g = e / nk;
  const int j = e - g * nk;
  const int r = rb + g;
  // row strides NH + 1: the lanes of a column tile read the same neuron of up to 16 rows, and
  // an NH-float4 stride put those rows 4 ways on the same LDS banks (PMC: ~1 conflict cycle
  // per LDS instruction, profiles/r4/pmc/final_pmc.md)
  const float4* recg = rec + g * (NH + 1);
  const float* hmg = hmx + g * (NH + 1);
  const float* bl = box + g * 2 * n0;
  const float sgn = s ? -1.f : 1.f;
  // lam = +-W_k[:, j] from the staged copy: element (in, j) of layer k's operand order
  float lam[TM][4];
  {
    const int jb = ((j >> 4) * 64 + 16 * ((j & 15) >> 2)) * 4 + (j & 3);
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // tiles t < the layer's input tiles are zero padded: load unguarded there
        const int in = 16 * t + 4 * grp + i;
        const float w = 16 * t < ktop ? wk[jb + (t * tk * 64 + 4 * grp + i) * 4] : 0.f;
        lam[t][i] = in < ktop ? sgn * w : 0.f;
      }
  }
  float c = sgn * smem[cfg.b_lds[k] + j];
  float err = 0.f;
  if constexpr (CS) {
    fa_refine_back_c<TM, WG, S, KC>(std::make_integer_sequence<int, KC>{}, net, cfg, smem, wsrc, recg, hmg, bl, n0,
                                    lane, u, lam, c, err);
  } else {
    for (int l = k - 1; l >= 0; --l)
      fa_refine_step<TM, WG, S, -1>(net, cfg, smem, wsrc, recg, hmg, bl, n0, lane, u, l, lam, c, err);
  }
  // ---- concretise over the row's box
  float cp = 0.f, mp = 0.f;
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    if (16 * t >= n0) break;                            // uniform
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int in = 16 * t + 4 * grp + i;
      if (TM <= 7) {   // clamped + select (10 tiles: the hoisted loads cost a wave per SIMD)
        const int ic = min(in, n0 - 1);
        const float xl = bl[ic], xh = bl[n0 + ic];
        const float lm = lam[t][i];
        const float dp = fminf(lm * xl, lm * xh), dm = fabsf(lm) * fmaxf(fabsf(xl), fabsf(xh));
        cp += in < n0 ? dp : 0.f;
        mp += in < n0 ? dm : 0.f;
      } else if (in < n0) {
        const float xl = bl[in], xh = bl[n0 + in];
        const float lm = lam[t][i];
        cp += fminf(lm * xl, lm * xh);
        mp += fabsf(lm) * fmaxf(fabsf(xl), fabsf(xh));
      }
    }
  }
  cp += __shfl_xor(cp, 16); cp += __shfl_xor(cp, 32);
  mp += __shfl_xor(mp, 16); mp += __shfl_xor(mp, 32);
  const float conc = cp + c;
  const float cmg = mp + fabsf(c);
  const float errK = err * (1.f + 2.f * gK);
  const float low = conc - errK - g0 * cmg - g1 * fabsf(conc);
  bool wr = vvalid;
  if (logit && wr && !cfg.full) {
    // REFINE + logit: replace the forward forms only where the backward ones concretise
    // tighter (both are sound; crown.hip's rule)
    wr = s ? (-low <= a.out_ub[r]) : (low >= a.out_lb[r]);
  }
  if (logit && wr) {
    // the logit's back-substituted forms: s = 0 lower (L), s = 1 upper (U = -form)
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int in = 16 * t + 4 * grp + i;
        if (in >= n0) continue;
        if (s) a.Uc[(size_t)r * n0 + in] = -lam[t][i];
        else a.Lc[(size_t)r * n0 + in] = lam[t][i];
      }
    if (grp == 0) {
      if (s) { a.U0[r] = -c; a.Ue[r] = errK; a.out_ub[r] = -low; }
      else { a.L0[r] = c; a.Le[r] = errK; a.out_lb[r] = low; }
    }
  }
  // lane group 0 of each column writes (the 4 groups hold the same column value)
  if (vvalid && grp == 0) {
    float* dst = slab + g * 2 * N + (s ? N : 0) + offk + j;
    *dst = s ? fminf(*dst, -low) : fmaxf(*dst, low);
    if (!logit && a.phase_in && a.infeas) {
      const int ph = a.phase_in[(size_t)r * NH + offk + j];
      if ((ph > 0 && s && -low < 0.f) || (ph < 0 && !s && low > 0.f)) a.infeas[r] = 1;
    }
  }
}

template <int TM, bool WG, class S, int... KS>
__device__ __forceinline__ void fa_refine_col_c(std::integer_sequence<int, KS...>, const NetDesc& net,
                                                const BoundArgs& a, const RefineCfg& cfg, const float* smem,
                                                const float* wsrc, float* slab, const float4* rec, const float* hmx,
                                                const float* box, const int* list, int k, int rb, int nv, int tile,
                                                int lane, float gK, float g0, float g1) {
  // k is wave-uniform: one compile-time column body per layer, selected by a scalar branch
  ((k == KS ? fa_refine_col<TM, WG, S, KS>(net, a, cfg, smem, wsrc, slab, rec, hmx, box, list, k, rb, nv, tile, lane,
                                           gK, g0, g1)
            : void()),
   ...);
}

// WG: the weights are read from the global backward-order block (NetDesc.wback_off; w_lds are
// offsets into it) instead of being staged: a 150-wide net's staged W (112 KB for BM-4) left LDS
// for one box row per workgroup.  A wave reads one float4 per lane per 8 MFMAs (256 cycles),
// ~4 B/clk, which L2 sustains for every wave of a CU.
template <int TM, bool WG = false, class S = FaShapeAny>
__global__ void __launch_bounds__(256) fa_refine_kernel(NetDesc net, BoundArgs a, RefineCfg cfg) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int L = net.n_layers;
  const int LW = (cfg.full || cfg.logit) ? L : L - 1;   // layers whose W is staged (+ the logit's)
  // ---- stage W_l (l < LW) in backward operand order + the biases
  for (int l = 0; l < LW; ++l) {
    const int nin = net.dims[l], nout = net.dims[l + 1];
    const int tin = (nin + 15) >> 4, tout = (nout + 15) >> 4;
    if (!WG) {
      const float* W = a.flat + net.w_off[l];
      float* dst = smem + cfg.w_lds[l];
      const int tot = tin * tout * 256;
      for (int e = tid; e < tot; e += 256) {
        const int i4 = e & 3, ln = (e >> 2) & 63, tt = e >> 8;
        const int t = tt % tout, ot = tt / tout;
        const int in = 16 * ot + (ln & 15), out = 16 * t + 4 * (ln >> 4) + i4;
        dst[e] = (in < nin && out < nout) ? W[(size_t)in * nout + out] : 0.f;
      }
    }
    for (int e = tid; e < nout; e += 256) smem[cfg.b_lds[l] + e] = a.flat[net.b_off[l] + e];
  }
  const float* wsrc = WG ? a.flat + net.wback_off : smem;
  const int lane = tid & 63, col = lane & 15, grp = lane >> 4;
  const int wave = tid >> 6;
  const int n0 = net.dims[0];
  const int N = net.n_neurons, NH = net.n_hidden;
  const float u = net.unit;
  const int G = cfg.G;
  float* slab = smem + cfg.slab;
  const float4* rec = reinterpret_cast<const float4*>(smem + cfg.rec);
  const float* hmx = smem + cfg.hm;
  float* box = smem + cfg.box;
  int* list = reinterpret_cast<int*>(smem + cfg.list);
  int* rrun = reinterpret_cast<int*>(smem + cfg.rrun);   // G running flags, then the column counter
  int K = 4 * L + 4;
  for (int l = 0; l < L; ++l) K += 2 * net.dims[l + 1];
  const float gK = fa_rgam(K, u);
  const float g0 = fa_rgam(n0 + 1, u);
  const float g1 = fa_rgam(1, u);
  for (int rb = blockIdx.x * G; rb < a.R; rb += gridDim.x * G) {
    __syncthreads();   // previous block's slab fully written back
    // ---- rows of running partitions (the others get no columns); skip the block if none
    if (tid < G) {
      const int r = rb + tid;
      int run = r < a.R;
      if (run && a.skip_status) {
        const int node = a.V > 0 ? r / a.V : r;
        const int8_t st = a.skip_status[a.skip_part[node]];
        run = (st == 3 || st == 4);
      }
      if (run && a.skip_signdef && cfg.logit && !cfg.full && a.V > 1) {
        // the forward bounds already close the node (sign shortcut over all ordered pairs)
        const int base = (r / a.V) * a.V;
        bool closed = true;
        for (int i = 0; i < a.V && closed; ++i)
          for (int j = 0; j < a.V; ++j)
            if (i != j && !(a.out_lb[base + i] >= 0.f || a.out_ub[base + j] <= 0.f)) { closed = false; break; }
        if (closed) run = 0;
      }
      rrun[tid] = run;
    }
    __syncthreads();
    bool any = false;
    for (int g = 0; g < G; ++g) any |= rrun[g] != 0;
    if (!any) continue;   // uniform across the workgroup (same LDS values everywhere)
    // ---- the rows' forward bounds (FULL: no forward pass, start from the whole line) and boxes
    // (protected attributes fixed to the row's values)
    for (int e = tid; e < G * N; e += 256) {
      const int g = e / N, k = e - g * N;
      const int r = min(rb + g, a.R - 1);
      slab[g * 2 * N + k] = cfg.full ? -INFINITY : a.layer_lb[(size_t)r * N + k];
      slab[g * 2 * N + N + k] = cfg.full ? INFINITY : a.layer_ub[(size_t)r * N + k];
    }
    for (int e = tid; e < G * n0; e += 256) {
      const int g = e / n0, d = e - g * n0;
      const int r = min(rb + g, a.R - 1);
      const int node = a.V > 0 ? r / a.V : r;
      const int v = a.V > 0 ? r - node * a.V : 0;
      float xl = a.lo[(size_t)node * n0 + d], xh = a.hi[(size_t)node * n0 + d];
      if (a.V > 0)
        for (int q = 0; q < a.npa; ++q)
          if (a.pa_idx[q] == d) xl = xh = a.values[v * a.npa + q];
      box[g * 2 * n0 + d] = xl;
      box[g * 2 * n0 + n0 + d] = xh;
    }
    __syncthreads();
    // REFINE starts at hidden layer 2: back-substituting a layer-1 neuron through layer 0 picks, per
    // weight sign, the same relaxation of h_0 the forward pass already combined (W+ U + W- L), so
    // its bounds only move by rounding (<= 4e-4 of the width, ops/reference.py:crown_refine) --
    // that layer was ~30 % of the kernel's column work on AC-7
    const int k0 = cfg.full ? 0 : 2, k1 = (cfg.full || cfg.logit) ? L : L - 1;
    if (!cfg.full)
      for (int l = 0; l < k0 && l < L - 1; ++l) fa_refine_records(net, a, cfg, l, rb, smem);   // final
    for (int k = k0; k < k1; ++k) {
      const bool logit = k == L - 1;               // the output forms (FULL, or REFINE + logit)
      const int nk = net.dims[k + 1];
      const int offk = net.neuron_off[k];
      // ---- the columns of this layer: both bounds of every UNSTABLE neuron of a running row (a
      // stable neuron's relaxation is exact whatever its interval, so tightening it buys nothing);
      // the logit: every running row
      if (tid == 0) rrun[G] = 0;
      __syncthreads();
      for (int e = tid; e < G * nk; e += 256) {
        const int g = e / nk, j = e - g * nk;
        bool take = rrun[g] != 0;
        if (take && !logit) {
          const float lb = slab[g * 2 * N + offk + j], ub = slab[g * 2 * N + N + offk + j];
          const uint8_t* dm = fa_refine_dmask(net, a, rb + g);
          // phase-fixed neurons too: a refined bound that contradicts the phase proves the node's
          // region empty (a.infeas)
          const bool fixed = a.phase_in && a.phase_in[(size_t)(rb + g) * NH + offk + j] != 0;
          // a dead-masked neuron outputs 0 whatever its bounds: REFINE skips it; FULL still bounds it
          // (its slab entries start at -inf / +inf and are written back like every other neuron's)
          take = ((lb < 0.f && ub > 0.f) || fixed) && !(dm && dm[offk + j] && !cfg.full);
        }
        if (take) list[atomicAdd(&rrun[G], 1)] = e;
      }
      __syncthreads();
      const int nv = 2 * rrun[G];
      const int ntile = (nv + 15) >> 4;
      for (int tile = wave; tile < ntile; tile += 4) {
        if constexpr (S::L > 0)
          fa_refine_col_c<TM, WG, S>(std::make_integer_sequence<int, S::L>{}, net, a, cfg, smem, wsrc, slab, rec, hmx,
                                     box, list, k, rb, nv, tile, lane, gK, g0, g1);
        else
          fa_refine_col<TM, WG, S, -1>(net, a, cfg, smem, wsrc, slab, rec, hmx, box, list, k, rb, nv, tile, lane, gK,
                                       g0, g1);
      }
      __syncthreads();
      if (k < L - 1) fa_refine_records(net, a, cfg, k, rb, smem);   // layer k is final now
    }
    // ---- write the refined hidden-layer bounds back (rows of running partitions only; FULL: only
    // when the caller wants them -- the BaB does not)
    if (cfg.full && !a.layer_lb) continue;
    const int lo_n = cfg.full ? 0 : net.neuron_off[1 < L - 1 ? 1 : 0];
    const int hi_n = cfg.full ? N : net.n_hidden;
    const int span = hi_n - lo_n;
    if (span > 0)
      for (int e = tid; e < G * span; e += 256) {
        const int g = e / span, k = lo_n + (e - (e / span) * span);
        if (!rrun[g]) continue;
        const int r = rb + g;
        a.layer_lb[(size_t)r * N + k] = slab[g * 2 * N + k];
        a.layer_ub[(size_t)r * N + k] = slab[g * 2 * N + N + k];
      }
  }
}

namespace {
typedef void (*RefineKernel)(NetDesc, BoundArgs, RefineCfg);
RefineKernel select_refine(int TM, bool wg) {
  if (TM <= 1) return fa_refine_kernel<1>;
  if (TM <= 2) return fa_refine_kernel<2>;
  if (TM <= 4) return fa_refine_kernel<4>;
  if (TM <= 7) return wg ? fa_refine_kernel<7, true> : fa_refine_kernel<7>;
  if (TM <= 10) return wg ? fa_refine_kernel<10, true> : fa_refine_kernel<10>;
  return nullptr;
}

// Compile-time shapes (common.h FaShape): the zoo's deep chains, each instantiated for the TM bucket
// select_refine picks for it (same LDS layout and arithmetic; the column body is unrolled per layer
// with constant widths).  FAIRIFY_REFINE_SHAPED=0 (read per launch: the bitwise-equality test toggles
// it) keeps the run-time-shape kernels.
struct ShapedRefine {
  int tm;
  bool wg;
  std::vector<int> dims;
  RefineKernel k;
};
template <int TM, int... D>
ShapedRefine shaped_refine() {
  return {TM, false, {D...}, fa_refine_kernel<TM, false, FaShape<D...>>};
}

RefineKernel select_refine_shaped(const NetDesc& net, int TM, bool wg) {
  const char* e = getenv("FAIRIFY_REFINE_SHAPED");
  if (e && *e == '0') return nullptr;
  static const std::vector<ShapedRefine> v = {
      shaped_refine<4, 13, 64, 32, 16, 8, 4, 1>(),    // AC-7
      shaped_refine<4, 16, 64, 32, 16, 8, 4, 1>(),    // BM-8
      shaped_refine<4, 13, 64, 64, 1>(),              // AC-5
      shaped_refine<7, 13, 100, 100, 1>(),            // AC-4
  };
  const int tmb = TM <= 1 ? 1 : TM <= 2 ? 2 : TM <= 4 ? 4 : TM <= 7 ? 7 : 10;
  for (const auto& s : v) {
    if (s.tm != tmb || s.wg != wg || (int)s.dims.size() != net.n_layers + 1) continue;
    bool same = true;
    for (int l = 0; l <= net.n_layers && same; ++l) same = s.dims[l] == net.dims[l];
    if (same) return s.k;
  }
  return nullptr;
}

// global-weights variant above this many staged bytes (FAIRIFY_REFINE_WG_KB: A/B and the
// bitwise-equality test; 0 = never; read per launch)
size_t refine_wg_bytes() {
  const char* e = getenv("FAIRIFY_REFINE_WG_KB");
  const long kb = e ? atol(e) : 64;
  return kb > 0 ? (size_t)kb * 1024 : (size_t)-1;
}

int refine_cus() {
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

namespace {
int backward_launch(const NetDesc& net, const BoundArgs& a, int full, int logit, hipStream_t stream) {
  const int L = net.n_layers;
  int TM = 1;
  for (int l = 0; l < L; ++l) TM = std::max(TM, (net.dims[l] + 15) / 16);
  RefineCfg cfg{};
  cfg.full = full;
  cfg.logit = logit;
  const int LW = (full || logit) ? L : L - 1;
  int offs = 0;
  for (int l = 0; l < LW; ++l) {
    cfg.w_lds[l] = offs;   // the LDS layout, and (WG) the same offsets in the global block
    offs += ((net.dims[l] + 15) / 16) * ((net.dims[l + 1] + 15) / 16) * 256;
  }
  const bool wg = (size_t)offs * sizeof(float) > refine_wg_bytes() && TM >= 5 && net.wback_floats >= offs;
  RefineKernel k = select_refine(TM, wg);
  if (!k) return -1;
  if (const RefineKernel ks = select_refine_shaped(net, TM, wg)) k = ks;
  if (wg) offs = 0;        // nothing staged: the biases start the LDS
  for (int l = 0; l < LW; ++l) {
    cfg.b_lds[l] = offs;
    offs += net.dims[l + 1];
  }
  const int base = (offs + 3) & ~3;
  const int N = net.n_neurons, NH = net.n_hidden, n0 = net.dims[0];
  int maxw = 1;
  for (int l = 1; l <= L; ++l) maxw = std::max(maxw, net.dims[l]);
  // per-row LDS: records 4 (NH + 1) (16-byte aligned, first), slab 2N, hm NH + 1, box 2 n0, columns maxw
  auto layout = [&](int g) {
    cfg.rec = base;
    cfg.slab = cfg.rec + g * 4 * (NH + 1);
    cfg.hm = cfg.slab + g * 2 * N;
    cfg.box = cfg.hm + g * (NH + 1);
    cfg.list = cfg.box + g * 2 * n0;
    cfg.rrun = cfg.list + g * maxw;
    return (size_t)(cfg.rrun + g + 1) * sizeof(float);
  };
  // rows per workgroup: 16 while two workgroups fit a CU's 160 KB (the VGPR budget allows two),
  // fewer for the widest nets, at least 1 within the 160 KB LDS
  static const size_t cap_bytes = [] {
    const char* e = getenv("FAIRIFY_REFINE_LDS_KB");   // A/B of the rows-per-workgroup rule
    return (size_t)(e ? atoi(e) : 80) * 1024;
  }();
  int G = 16;
  while (G > 1 && layout(G) > cap_bytes) G /= 2;
  if (layout(G) > 160 * 1024) return -1;
  cfg.G = G;
  const size_t bytes = layout(G);
  cfg.floats = (int)(bytes / sizeof(float));
  if (!fa_lds_ok(bytes)) return -4;
  static std::mutex mu;
  static std::map<std::pair<const void*, size_t>, int> occ;
  int per_cu = 0;
  {
    std::lock_guard<std::mutex> g(mu);
    const auto key = std::make_pair((const void*)k, bytes);
    auto it = occ.find(key);
    if (it == occ.end()) {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256, bytes) != hipSuccess || per_cu <= 0) per_cu = 1;
      occ[key] = per_cu;
    } else {
      per_cu = it->second;
    }
  }
  long long blocks = ((long long)a.R + G - 1) / G;
  const long long cap = (long long)refine_cus() * per_cu * 4;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(256), bytes, stream, net, a, cfg);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e - 10;
}
}  // namespace

// 0 launched (or nothing to refine: fewer than two hidden layers), -1 shape not supported (a layer
// wider than 160 or the weights beyond the LDS budget: the caller keeps the forward bounds, which
// are sound), < -1 error.  Needs a.layer_lb / a.layer_ub [R, n_neurons] from the forward pass.
extern "C" int fa_refine_launch(const NetDesc& net, BoundArgs a, hipStream_t stream) {
  if (a.R <= 0 || net.n_layers < 4) return 0;   // refines hidden layers 2 .. L-2
  if (!a.layer_lb || !a.layer_ub) return -2;
  return backward_launch(net, a, 0, 0, stream);
}

// REFINE + the logit's backward pass in the same launch (replaces fa_refine_launch + fa_crown_launch):
// out_lb / out_ub and the forms of a preceding forward pass are tightened in place.
extern "C" int fa_refine_crown_launch(const NetDesc& net, BoundArgs a, hipStream_t stream) {
  if (a.R <= 0) return 0;
  if (net.n_layers < 3) return -1;
  if (!a.layer_lb || !a.layer_ub || !a.out_lb || !a.Lc || !a.Uc) return -2;
  return backward_launch(net, a, 0, 1, stream);
}

// Mode FULL: out_lb / out_ub and the logit's forms (Lc, L0, Le, Uc, U0, Ue) of every row without a
// forward pass; layer_lb / layer_ub [R, n_neurons] written when given.  0 launched, -1 shape not
// supported (the caller runs the forward pass instead), < -1 error.
extern "C" int fa_backward_launch(const NetDesc& net, BoundArgs a, hipStream_t stream) {
  if (a.R <= 0) return 0;
  if (!a.out_lb || !a.out_ub || !a.Lc || !a.L0 || !a.Le || !a.Uc || !a.U0 || !a.Ue) return -2;
  return backward_launch(net, a, 1, 1, stream);
}

FA_LDS_REGISTER(FA_LDS_K((fa_refine_kernel<7, true>)), FA_LDS_K((fa_refine_kernel<10, true>)));
FA_LDS_REGISTER(FA_LDS_K(fa_refine_kernel<1>), FA_LDS_K(fa_refine_kernel<2>), FA_LDS_K(fa_refine_kernel<4>),
                FA_LDS_K(fa_refine_kernel<7>), FA_LDS_K(fa_refine_kernel<10>));
FA_LDS_REGISTER(FA_LDS_K((fa_refine_kernel<4, false, FaShape<13, 64, 32, 16, 8, 4, 1>>)),
                FA_LDS_K((fa_refine_kernel<4, false, FaShape<16, 64, 32, 16, 8, 4, 1>>)),
                FA_LDS_K((fa_refine_kernel<4, false, FaShape<13, 64, 64, 1>>)),
                FA_LDS_K((fa_refine_kernel<7, false, FaShape<13, 100, 100, 1>>)));
