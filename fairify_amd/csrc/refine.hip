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
// per tile).
#include <hip/hip_runtime.h>

#include <stdlib.h>

#include <algorithm>
#include <map>
#include <mutex>

#include "args.h"

// Mode FULL (fa_backward_launch): no forward pass at all -- layer 0 from the box, every hidden layer
// by back-substitution, then the logit's forms and bounds (the work of crown.hip) in the same
// launch: one kernel instead of forward symbolic + refine + output pass (ops/reference.py:
// backward_bounds).  Mode REFINE (fa_refine_launch): tighten the forward pass's hidden-layer bounds.
struct RefineCfg {
  int w_lds[FA_MAX_LAYERS];   // LDS float offset of layer l's W in backward operand order
  int b_lds[FA_MAX_LAYERS];
  int slab;                   // LDS float offset of the row slabs: G x [lb (N) | ub (N)]
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

template <int TM>
__global__ void __launch_bounds__(256) fa_refine_kernel(NetDesc net, BoundArgs a, RefineCfg cfg) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int L = net.n_layers;
  const int LW = (cfg.full || cfg.logit) ? L : L - 1;   // layers whose W is staged (+ the logit's)
  // ---- stage W_l (l < LW) in backward operand order + the biases
  for (int l = 0; l < LW; ++l) {
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
  const int lane = tid & 63, col = lane & 15, grp = lane >> 4;
  const int wave = tid >> 6;
  const int n0 = net.dims[0];
  const int N = net.n_neurons;
  const float u = net.unit;
  const int G = cfg.G;
  float* slab = smem + cfg.slab;
  int K = 4 * L + 4;
  for (int l = 0; l < L; ++l) K += 2 * net.dims[l + 1];
  const float gK = fa_rgam(K, u);
  const float g0 = fa_rgam(n0 + 1, u);
  const float g1 = fa_rgam(1, u);
  for (int rb = blockIdx.x * G; rb < a.R; rb += gridDim.x * G) {
    __syncthreads();   // previous block's slab fully written back
    // ---- block-uniform skip: every row of the block invalid or of a decided partition
    bool any = false;
    for (int g = 0; g < G && !any; ++g) {
      const int r = rb + g;
      if (r >= a.R) break;
      if (!a.skip_status) { any = true; break; }
      const int node = a.V > 0 ? r / a.V : r;
      const int8_t st = a.skip_status[a.skip_part[node]];
      any = (st == 3 || st == 4);
    }
    if (!any) continue;   // uniform across the workgroup (same loads everywhere)
    // ---- load the rows' forward bounds (FULL: no forward pass, start from the whole line)
    for (int e = tid; e < G * N; e += 256) {
      const int g = e / N, k = e - g * N;
      const int r = min(rb + g, a.R - 1);
      slab[g * 2 * N + k] = cfg.full ? -INFINITY : a.layer_lb[(size_t)r * N + k];
      slab[g * 2 * N + N + k] = cfg.full ? INFINITY : a.layer_ub[(size_t)r * N + k];
    }
    __syncthreads();
    const int k0 = cfg.full ? 0 : 1, k1 = (cfg.full || cfg.logit) ? L : L - 1;
    for (int k = k0; k < k1; ++k) {
      const bool logit = k == L - 1;               // the output forms (FULL, or REFINE + logit)
      const int nk = net.dims[k + 1];
      const int ktop = net.dims[k];                  // width of h_{k-1}
      const int offk = net.neuron_off[k];
      const int nv = G * 2 * nk;
      const int ntile = (nv + 15) >> 4;
      const float* Wk = a.flat + net.w_off[k];
      for (int tile = wave; tile < ntile; tile += 4) {
        const int idx0 = tile * 16 + col;
        const bool vvalid = idx0 < nv;
        const int idx = vvalid ? idx0 : nv - 1;
        const int g = idx / (2 * nk);
        const int rem = idx - g * 2 * nk;
        const int s = rem / nk;
        const int j = rem - s * nk;
        const int r0 = rb + g;
        const bool rvalid = vvalid && r0 < a.R;
        const int r = min(r0, a.R - 1);
        const int node = a.V > 0 ? r / a.V : r;
        const int v = a.V > 0 ? r - node * a.V : 0;
        const uint8_t* dmask = nullptr;
        if (a.dead_in) dmask = a.dead_in + (size_t)r * net.n_hidden;
        else if (a.dead_part)
          dmask = a.dead_part + (size_t)a.node_part[a.part_mod ? node % a.part_mod : node] * net.n_hidden;
        const float* lbr = slab + g * 2 * N;
        const float* ubr = lbr + N;
        const float sgn = s ? -1.f : 1.f;
        float lam[TM][4];
#pragma unroll
        for (int t = 0; t < TM; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int in = 16 * t + 4 * grp + i;
            lam[t][i] = in < ktop ? sgn * Wk[(size_t)in * nk + j] : 0.f;
          }
        float c = sgn * smem[cfg.b_lds[k] + j];
        float err = 0.f;
        for (int l = k - 1; l >= 0; --l) {
          const int n = net.dims[l + 1];
          const int nin = net.dims[l];
          const int tout = (n + 15) >> 4, tin = (nin + 15) >> 4;
          const int off = net.neuron_off[l];
          const float* b = smem + cfg.b_lds[l];
          float mu[TM][4];
          float cs = 0.f, cm = 0.f, er = 0.f;
#pragma unroll
          for (int t = 0; t < TM; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int jj = 16 * t + 4 * grp + i;
              const bool jv = t < tout && jj < n;
              const float lb = jv ? lbr[off + jj] : 0.f, ub = jv ? ubr[off + jj] : 0.f;
              const bool dd = !jv || ub <= 0.f || (dmask && dmask[off + jj]);
              const bool act = !dd && lb >= 0.f;
              const bool unst = !dd && !act;
              const float alpha = ub > -lb ? 1.f : 0.f;
              const float sl = unst ? (ub / (ub - lb)) * (1.f + 4.f * u) : 0.f;
              const float zmax = fmaxf(fabsf(lb), fabsf(ub));
              const float bj = jv ? b[jj] : 0.f;
              const float lm = lam[t][i];
              const float slope = act ? 1.f : (dd ? 0.f : (lm >= 0.f ? alpha : sl));
              const float m = lm * slope;
              const bool neg = unst && lm < 0.f;
              const float tt = neg ? -m * lb : 0.f;
              mu[t][i] = m;
              cs += m * bj + tt;
              cm += fabsf(m * bj) + fabsf(tt);
              if (neg) er += 3.f * u * (fabsf(m) * zmax + fabsf(tt));
            }
          const float4* wb = reinterpret_cast<const float4*>(smem + cfg.w_lds[l]);
          const float gn = fa_rgam(2 * n + 1, u);
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
              float hm = 0.f;
              if (in < nin) {
                if (l > 0) {
                  const int po = net.neuron_off[l - 1];
                  hm = fmaxf(ubr[po + in], 0.f);
                  if (dmask && dmask[po + in]) hm = 0.f;
                } else {
                  float xl = a.lo[(size_t)node * n0 + in], xh = a.hi[(size_t)node * n0 + in];
                  if (a.V > 0)
                    for (int q = 0; q < a.npa; ++q)
                      if (a.pa_idx[q] == in) xl = xh = a.values[v * a.npa + q];
                  hm = fmaxf(fabsf(xl), fabsf(xh));
                }
              }
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
        // ---- concretise over the row's box
        float cp = 0.f, mp = 0.f;
#pragma unroll
        for (int t = 0; t < TM; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int in = 16 * t + 4 * grp + i;
            if (in >= n0) continue;
            float xl = a.lo[(size_t)node * n0 + in], xh = a.hi[(size_t)node * n0 + in];
            if (a.V > 0)
              for (int q = 0; q < a.npa; ++q)
                if (a.pa_idx[q] == in) xl = xh = a.values[v * a.npa + q];
            const float lm = lam[t][i];
            cp += fminf(lm * xl, lm * xh);
            mp += fabsf(lm) * fmaxf(fabsf(xl), fabsf(xh));
          }
        cp += __shfl_xor(cp, 16); cp += __shfl_xor(cp, 32);
        mp += __shfl_xor(mp, 16); mp += __shfl_xor(mp, 32);
        const float conc = cp + c;
        const float cmg = mp + fabsf(c);
        const float errK = err * (1.f + 2.f * gK);
        const float low = conc - errK - g0 * cmg - g1 * fabsf(conc);
        bool wr = rvalid;
        if (logit && wr && a.skip_status) {       // forms of decided partitions' rows: not needed
          const int8_t st = a.skip_status[a.skip_part[node]];
          wr = (st == 3 || st == 4);
        }
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
        if (rvalid && grp == 0) {
          float* dst = slab + g * 2 * N + (s ? N : 0) + offk + j;
          *dst = s ? fminf(*dst, -low) : fmaxf(*dst, low);
        }
      }
      __syncthreads();
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
        const int r = rb + g;
        if (r >= a.R) continue;
        if (a.skip_status) {
          const int node = a.V > 0 ? r / a.V : r;
          const int8_t st = a.skip_status[a.skip_part[node]];
          if (!(st == 3 || st == 4)) continue;
        }
        a.layer_lb[(size_t)r * N + k] = slab[g * 2 * N + k];
        a.layer_ub[(size_t)r * N + k] = slab[g * 2 * N + N + k];
      }
  }
}

namespace {
typedef void (*RefineKernel)(NetDesc, BoundArgs, RefineCfg);
RefineKernel select_refine(int TM) {
  if (TM <= 1) return fa_refine_kernel<1>;
  if (TM <= 2) return fa_refine_kernel<2>;
  if (TM <= 4) return fa_refine_kernel<4>;
  if (TM <= 7) return fa_refine_kernel<7>;
  if (TM <= 10) return fa_refine_kernel<10>;
  return nullptr;
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
  const RefineKernel k = select_refine(TM);
  if (!k) return -1;
  RefineCfg cfg{};
  cfg.full = full;
  cfg.logit = logit;
  const int LW = (full || logit) ? L : L - 1;
  int offs = 0;
  for (int l = 0; l < LW; ++l) {
    cfg.w_lds[l] = offs;
    offs += ((net.dims[l] + 15) / 16) * ((net.dims[l + 1] + 15) / 16) * 256;
  }
  for (int l = 0; l < LW; ++l) {
    cfg.b_lds[l] = offs;
    offs += net.dims[l + 1];
  }
  cfg.slab = (offs + 3) & ~3;
  const int N = net.n_neurons;
  // rows per workgroup: 16 when the slab fits next to the weights in 64 KB (2+ workgroups per CU),
  // fewer for the widest nets, at least 1 within the 160 KB LDS
  int G = 16;
  auto bytes_for = [&](int g) { return ((size_t)cfg.slab + (size_t)g * 2 * N) * sizeof(float); };
  while (G > 1 && bytes_for(G) > 64 * 1024) G /= 2;
  if (bytes_for(G) > 160 * 1024) return -1;
  cfg.G = G;
  cfg.floats = cfg.slab + G * 2 * N;
  const size_t bytes = bytes_for(G);
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
  if (a.R <= 0 || net.n_layers < 3) return 0;
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

FA_LDS_REGISTER(FA_LDS_K(fa_refine_kernel<1>), FA_LDS_K(fa_refine_kernel<2>), FA_LDS_K(fa_refine_kernel<4>),
                FA_LDS_K(fa_refine_kernel<7>), FA_LDS_K(fa_refine_kernel<10>));
