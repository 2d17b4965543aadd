// Register-resident forward-symbolic bound propagation (K4/K9 bounding primitive).  gfx950.
//
// Same arithmetic and error accounting as fa_bounds_kernel / ops/reference.py:bounds (symbolic
// mode), re-tiled for CDNA4:
//
// * ONE box-row per wave64 (many waves per CU, persistent grid), no __syncthreads after the
//   one-time staging of every layer's W and b into LDS.
// * A layer's linear forms are kept TRANSPOSED in MFMA accumulators: rows = neurons, columns =
//   form columns [coefficients of the non-folded input dims | constant | error | interval |
//   interval error].  Input dims that are degenerate for every row (the protected attribute
//   in the node-row expansion, V > 0) are folded into the constant column, so Adult's
//   13-input forms (12 coefficients + 4) fill exactly one 16-wide column tile.
// * Layer l is   U' = W+^T U + W-^T L,   L' = W+^T L + W-^T U   on v_mfma_f32_16x16x4_f32.
//   The L block stores its two error columns NEGATED, so the same four plain MFMAs make both
//   error columns accumulate |W-| (U_err' = W+ eU + |W-| eL, -L_err' = -(W+ eL + |W-| eU)).
//   The previous layer's accumulator tile IS the next layer's B operand (reg i of tile t holds
//   neurons 16t + 4*(lane>>4) + i); W^T is staged in LDS pre-permuted into that MFMA operand
//   order, one ds_read_b128 per (output tile, K tile), so forms never touch LDS or HBM
//   between layers.
// * The epilogue works on the accumulators: constant/error/interval columns are broadcast and
//   the concretisation sums reduced within each 16-lane row with DPP (quad_perm, row
//   half-mirror, row mirror: a butterfly, so every lane holds the bitwise-identical sum), and
//   the ReLU relaxation rescales each lane's own column.
//
// Shapes outside the register budget (wide layers with > 1 column tile) keep using the
// LDS-tiled fa_bounds_kernel; see fa_sym_try_launch.
#include <hip/hip_runtime.h>

#include <stdlib.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <tuple>
#include <utility>
#include <vector>

#include "args.h"

#define FA_SYM_MAXC 48   // at most 3 column tiles

struct SymCfg {
  int nc;                          // coefficient columns (non-folded input dims)
  int cdim[FA_SYM_MAXC];           // column -> input dim (c < nc)
  unsigned long long fold;         // bitmask of folded (degenerate) input dims
  int w_lds[FA_MAX_LAYERS];        // LDS float offset of W_l, MFMA operand order:
                                   //   [jt][t][lane][i] = W[16t + 4(lane>>4) + i][16jt + (lane&15)]
  int b_lds[FA_MAX_LAYERS];        // LDS float offset of b_l
  int lds_floats;
  int stage_off;                   // float offset in `flat` of the staged block (wperm or packed)
  int stage_floats;                //   and its size (multiple of 4)
};

// Compile-time network shape (common.h FaShape) for the zoo shapes that dominate the bench and the
// big grids.  With the shape known, the layer loop is unrolled at compile time (fa_sym_layers_c):
// every per-layer width, tile count, "last layer" test and partial-tile lane mask is a constant,
// so the tile loops lose their uniform trip-count checks and the epilogue its width guards -- the
// scalar work the PMC pass charged to these kernels (SALU:VALU 0.34-0.44, profiles/r5/pmc_diet.md).
// SymShapeAny (L = 0): widths read from NetDesc at run time, any network.
using SymShapeAny = FaShapeAny;
template <int... D>
using SymShape = FaShape<D...>;

struct SymBox {
  const BoundArgs* a;
  int node, v, n0;
  __device__ __forceinline__ float lo(int d) const {
    float x = a->lo[(size_t)node * n0 + d];
    if (a->V > 0)
      for (int k = 0; k < a->npa; ++k)
        if (a->pa_idx[k] == d) x = a->values[v * a->npa + k];
    return x;
  }
  __device__ __forceinline__ float hi(int d) const {
    float x = a->hi[(size_t)node * n0 + d];
    if (a->V > 0)
      for (int k = 0; k < a->npa; ++k)
        if (a->pa_idx[k] == d) x = a->values[v * a->npa + k];
    return x;
  }
};

// Row rotation of the epilogue's staging tile: form column c of tile row rho (0..31: 16 U rows, 16
// L rows) sits at rho * TS + c + (rho >> 3).  The spill / reload (lanes of one 32-lane half write
// or read 2 rows that share rho >> 3, 16 consecutive columns each) stay conflict-free as with the
// plain layout (TS = 4 mod 8), and the per-lane row walk of the epilogue -- 32 lanes on 32
// different rows, the compiler splits it into ds_read2_b32 / ds_write2_b32 pairs (banks mod 32) --
// no longer hits the 8-row period of the 20-float stride: rows rho and rho + 8 land 1 bank apart
// instead of on the same bank (4-way conflicts, 1.7-1.9 conflict cycles per LDS instruction in
// profiles/r3/pmc/README.md).  Columns stay below TS: c <= 16 NT - 1, shift <= 3, TS = 16 NT + 4.
__device__ __forceinline__ int fa_trot(int rho) { return rho >> 3; }

// per-wave LDS slab: tile staging T[2 blocks][16 neurons][TS] + box values [2 PG boxes][3][48]
// (+ packed mode: the boxes' input ranges [2 PG][lo 16 | hi 16] for the on-the-fly layer-0 operands)
template <int NT, int PG = 1>
struct SymSlab {   // box values per column: [mid | rad | m] x FA_SYM_MAXC
  static constexpr int TS = 16 * NT + 4;                 // padded row stride (floats)
  static constexpr int TILE1 = 2 * 16 * TS;             // one 16-neuron tile, U and L blocks
  static constexpr int TILE = 2 * TILE1;                 // two tiles per epilogue pass
  static constexpr int BOX = 3 * FA_SYM_MAXC;
  static constexpr int BOXTAB = PG > 1 ? 2 * PG * 32 : 0;
  static constexpr int FLOATS = (TILE + 2 * PG * BOX + BOXTAB + 3) & ~3;
};

// Epilogue of one 16-neuron output tile (accumulators U, Lq of tile jt): spill to the wave's
// LDS slab, one lane per (neuron, block) computes the rigorous bounds and the ReLU relaxation
// once, the new form rows are reloaded in MFMA operand layout into (nu, nlo).  Returns false on
// the last layer (outputs written, nothing to reload).
//
// Packed mode (PG > 1, narrow networks): tile row `col` of group tsub is neuron col % S of box
// tsub * PG + col / S of the wave pass, S = 16 / PG (a multiple of 4, so a box's K terms fill
// the MFMA K steps exactly as in the unpacked kernel: bitwise the same bounds whatever boxes
// share the tile); rows j >= the layer's width are padding; the wave's boxes are consecutive
// rows r_in + b.
// Centre / radius layer GEMM (multi-tile kernels, FA_SYM_CR): the operands of a layer are
// C = (U + L) / 2 and R = (U - L) / 2 of the previous layer's upper / lower rows (L rows carry
// their error columns negated), so  U' = W+ U + W- L = W C + |W| R  and  L' = W C - |W| R:  two
// MFMA chains (P = W C, Q = |W| R; |w| is a free source modifier) instead of four.  Rounding:
// every output term passes through at most n_in + 2 roundings (C/R formation, the n_in-term
// chain, P +- Q); the error columns recombine W+ eU + |W-| eL from (eU - eL)/2 and (eU + eL)/2,
// so their rounding is bounded by 2 gamma Q (added once more on columns 1 and 3), and each input
// row's error columns carry the rounding budget of BOTH blocks (gamma (m_U + m_L),
// gamma max(iv_U, iv_L)): the radius couples them.
//
// The coupling costs exactness: a lower row that is exactly zero (dead neuron, lambda = 0) picks
// up the upper row's rounding budget.  Narrow random-init nets decide many partitions through an
// exactly zero logit, and the C/R form on the paired / packed kernels cost the bench 6.3 points
// of verified partitions (profiles/r2/s4/README.md), so only the multi-tile kernels (wide
// layers, where an all-dead layer does not occur) use it.
template <bool PAIR, int TM>
struct SymForm {
  static constexpr bool CR = !PAIR && TM >= 2;
};

// fc = FORM column of the lane (ct * 16 + (lane & 15)): only the two error columns (1 and 3 of
// column tile 0) carry the recombination slack; a coefficient column of a later tile with the same
// lane index must not move (round-2 advisor finding: +-e on coefficient columns 17 / 19 shifted
// the forms instead of widening them)
__device__ __forceinline__ void fa_pq_to_ul(const f32x4& P, const f32x4& Q, int fc, float gg, f32x4& U,
                                            f32x4& L) {
  const float sl = (fc == 1 || fc == 3) ? 2.f * gg : 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float q = Q[i], e = sl * fabsf(q);
    U[i] = (P[i] + q) + e;
    L[i] = (P[i] - q) - e;
  }
}

template <int NT, bool PAIR, int PG = 1, bool CR = false, class S = SymShapeAny>
__device__ __forceinline__ bool fa_sym_epilogue(const NetDesc& net, const BoundArgs& a, const SymCfg& cfg,
                                                const float* smem, float* T, const float* bxv_in, const int* cdim_s,
                                                int l, int r_in, int node_in, int r2, int node2, bool v2, int lane,
                                                int jt0, const f32x4 (&U)[2][NT],
                                                const f32x4 (&Lq)[2][NT], float (&nu)[2][NT][4],
                                                float (&nlo)[2][NT][4]) {
  constexpr int TS = SymSlab<NT>::TS;
  constexpr bool CS = S::L > 0;        // compile-time shape: l is a constant here (fa_sym_layers_c)
  const int col = lane & 15, grp = lane >> 4;
  const int n_out = CS ? S::dim(l + 1) : net.dims[l + 1];
  const float* sb = smem + cfg.b_lds[l];
  const bool last = CS ? l == S::L - 1 : l == net.n_layers - 1;
  const float gg = net.g_gemm[l];
  const float gc = net.g_conc;
  const float gi = net.g_one;
  const float unit = net.unit;
  // next layer's rounding budget; C/R: gamma_{n_in + 3} (n_in + 2 roundings), charged on both blocks
  const float gnext = last ? 0.f : (CR ? net.g_fwd[l + 1] : net.g_gemm[l + 1]);
  const int noff = net.neuron_off[l];
  const int nc = cfg.nc;
  const int n0 = CS ? S::dim(0) : net.dims[0];
  // neuron lane role in the epilogue: tile jt0 + (lane >> 5); within it lanes 0-15 = U block,
  // 16-31 = L block of neuron (lane & 15) -- all 64 lanes busy for two output tiles.  PAIR: the
  // two tiles are the same neurons of two box rows (r_in, r2), each with its own box values
  const int tsub = lane >> 5;
  const bool second = PAIR && tsub;
  constexpr int PS = 16 / PG;                            // packed: rows per box
  const int gbox = PG > 1 ? col / PS : 0;                // packed: box of this tile row in its group
  const int bidx = tsub * PG + gbox;                     // packed: box index within the wave pass
  const int r = PG > 1 ? r_in + bidx : (second ? r2 : r_in);
  const int node = PG > 1 ? (a.V > 0 ? r / a.V : r) : (second ? node2 : node_in);
  const float* bxv = bxv_in + (PG > 1 ? bidx : (second ? 1 : 0)) * SymSlab<NT, PG>::BOX;
  const int jt = PAIR ? jt0 : jt0 + tsub;
  const int n_out_t = n_out;
  const bool nl_act = PG > 1 ? r < a.R : (16 * jt < n_out_t && (!second || v2));
  const int ob = (lane >> 4) & 1;
  // this lane's row (tile row ob * 16 + col of tile tsub), rotated (fa_trot)
  float* Trow = T + tsub * SymSlab<NT>::TILE1 + (ob * 16 + col) * TS + fa_trot(ob * 16 + col);
    // ---------------- spill both tiles: T[tile][block][neuron][column] (rotated rows)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ru = 4 * grp + i, rl = 16 + 4 * grp + i;
          T[u * SymSlab<NT>::TILE1 + ru * TS + fa_trot(ru) + ct * 16 + col] = U[u][ct][i];
          T[u * SymSlab<NT>::TILE1 + rl * TS + fa_trot(rl) + ct * 16 + col] = Lq[u][ct][i];
        }
    __builtin_amdgcn_wave_barrier();
    // ---------------- one lane per (tile, neuron, block): bounds, relaxation, new form row
    const int j = PG > 1 ? col - gbox * PS : 16 * jt + col;   // neuron within its box
    const bool jv = j < n_out;
    float v[16 * NT];
#pragma unroll
    for (int c = 0; c < 16 * NT; ++c) v[c] = Trow[c];
    // packed biases: 16 per layer, box g at g * PS; clamped index + select (a guarded load is an
    // exec-mask branch)
    const float braw = sb[PG > 1 ? col : min(j, n_out - 1)];
    const float b = jv ? braw : 0.f;
    // concretisation of the coefficient part over the box in centre/radius form:
    //   min / max = Σ v mid -+ Σ |v| rad,  magnitude Σ |v| m  (m >= |mid| + rad)
    // three FMAs per column (|v| is a free source modifier) instead of two products, a min, a max
    // and three adds; rounding: Σ v mid and Σ |v| rad carry gamma_nc each and the final
    // subtraction / constant add two more roundings, within the gamma_{n0+3} of g_conc times the
    // magnitude.  Padding columns hold 0 coefficients and a 0 box: exact zeros.
    float s1 = 0.f, s2 = 0.f, mg = 0.f;
#pragma unroll
    for (int c = 4; c < 16 * NT; ++c) {
      const float av = fabsf(v[c]);
      s1 = fmaf(v[c], bxv[c], s1);
      s2 = fmaf(av, bxv[FA_SYM_MAXC + c], s2);
      mg = fmaf(av, bxv[2 * FA_SYM_MAXC + c], mg);
    }
    float mn = s1 - s2, mx = s1 + s2;
    const float cr = v[0];
    float er = v[1], ivr = v[2], ier = v[3];
    const float sgn = ob ? -1.f : 1.f;            // L block: error columns stored negated
    er *= sgn;
    ier *= sgn;
    const float c0 = cr + b;
    const float mgc = mg;                         // coefficient part of the magnitude
    mn += c0; mx += c0; mg += fabsf(c0);
    const float iv = ivr + b;
    const float eI = ier * (1.f + 2.f * gg) + gg * fabsf(b);
    const float e = er * (1.f + 2.f * gg) + gg * fabsf(b);
    float bound;
    if (ob == 0) bound = fminf(iv + gi * fabsf(iv) + eI, mx + gc * mg + e);   // ub (U block)
    else bound = fmaxf(iv - gi * fabsf(iv) - eI, mn - gc * mg - e);           // lb (L block)
    const float other = __shfl_xor(bound, 16, 64);
    const float ub = ob == 0 ? bound : other;
    const float lb = ob == 0 ? other : bound;
    if (nl_act && jv && a.layer_lb) {
      if (ob == 0) a.layer_ub[(size_t)r * net.n_neurons + noff + j] = ub;
      else a.layer_lb[(size_t)r * net.n_neurons + noff + j] = lb;
    }
    if (last) {
      if (nl_act && j == 0) {   // logit: rigorous bounds + output forms (folded dims -> 0)
        float* Cf = ob == 0 ? a.Uc : a.Lc;
        if (ob == 0) {
          a.out_ub[r] = ub; a.U0[r] = c0; a.Ue[r] = e;
        } else {
          a.out_lb[r] = lb; a.L0[r] = c0; a.Le[r] = e;
        }
        for (int d = 0; d < n0; ++d)
          if ((cfg.fold >> d) & 1ull) Cf[(size_t)r * n0 + d] = 0.f;
        for (int c = 0; c < nc; ++c) Cf[(size_t)r * n0 + cdim_s[c]] = Trow[4 + c];
      }
      return false;
    }
    bool forced = false, fact = false;
    if (nl_act && jv) {
      if (a.dead_in) forced = a.dead_in[(size_t)r * net.n_hidden + noff + j] != 0;
      else if (a.dead_part) forced = a.dead_part[(size_t)a.node_part[node] * net.n_hidden + noff + j] != 0;
      if (a.phase_in) {   // ReLU-phase rows: fixed inactive = forced dead, fixed active = no chord
        const int8_t ph = a.phase_in[(size_t)r * net.n_hidden + noff + j];
        forced = forced || ph < 0;
        fact = ph > 0;
        if (ob == 0 && a.infeas && ((ph < 0 && lb > 0.f) || (ph > 0 && ub < 0.f))) a.infeas[r] = 1;
      }
    }
    const bool isdead = ub <= 0.f;
    const bool isact = lb >= 0.f;
    if (nl_act && ob == 0 && jv && a.dead_out) a.dead_out[(size_t)r * net.n_hidden + noff + j] = isdead ? 1 : 0;
    const bool zero = isdead || forced || !jv;
    // both blocks' relaxations, then a per-lane select: the U and L lanes share every wave, so
    // a branch on ob runs both sides anyway, plus the exec-mask juggling (SALU)
    //   upper: identity (stable active, or the upper form T = U + eU >= 0 on the whole box:
    //   relu(z) <= T there, a chord from (aa, 0) would cut below it) / zero / chord over [aa, bb]
    const float aa = mn - gc * mg + e;
    const float bb = mx + gc * mg + e;
    const bool chord = !zero && !isact && !fact && aa < 0.f;
    const float sc = (bb / (bb - aa)) * (1.f + 4.f * unit);     // used only where chord
    const float shift = e - aa;
    const float cc = c0 * sc + sc * shift;
    const float sU = zero ? 0.f : (chord ? sc : 1.f);
    const float cU = zero ? 0.f : (chord ? cc : c0);
    const float mU = zero ? 0.f : (chord ? sc * mgc * (1.f + 8.f * unit) + fabsf(cc) : mg);
    const float eU = zero ? 0.f : (chord ? 4.f * unit * sc * (mg + fabsf(shift)) : e);
    //   lower: lambda in {0,1} applied to L(x) - eL
    const float aL = mn - gc * mg - e;
    const float bL = mx + gc * mg - e;
    const bool lam1 = !zero && (isact || ((bL > 0.f) && (bL > -aL)));
    const bool up = ob == 0;
    const float ivn = zero ? 0.f : fmaxf(up ? ub : lb, 0.f);
    const float s = up ? sU : (lam1 ? 1.f : 0.f);
    const float cnew = up ? cU : (lam1 ? c0 : 0.f);
    const float en = up ? eU : (lam1 ? e : 0.f);
    const float mgn = up ? mU : (lam1 ? mg : 0.f);
    // new row: constant, error, interval, interval error (L errors negated), scaled coefficients
    const float mg_b = CR ? mgn + __shfl_xor(mgn, 16, 64) : mgn;            // C/R: both blocks
    const float iv_b = CR ? fmaxf(ivn, __shfl_xor(ivn, 16, 64)) : ivn;
    v[0] = cnew;
    v[1] = sgn * (en + gnext * mg_b);
    v[2] = ivn;
    v[3] = sgn * (gnext * iv_b);
#pragma unroll
    for (int c = 4; c < 16 * NT; ++c) v[c] *= s;
    if (nl_act) {
#pragma unroll
      for (int c = 0; c < 16 * NT; ++c) Trow[c] = v[c];
    }
    __builtin_amdgcn_wave_barrier();
    // ---------------- reload both tiles in MFMA operand layout: next layer's B
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ru = 4 * grp + i, rl = 16 + 4 * grp + i;
          const float xu = T[u * SymSlab<NT>::TILE1 + ru * TS + fa_trot(ru) + ct * 16 + col];
          const float xl = T[u * SymSlab<NT>::TILE1 + rl * TS + fa_trot(rl) + ct * 16 + col];
          nu[u][ct][i] = CR ? 0.5f * (xu + xl) : xu;     // C/R: centre / radius operands
          nlo[u][ct][i] = CR ? 0.5f * (xu - xl) : xl;
        }
    __builtin_amdgcn_wave_barrier();
    return true;
}

// PAIR (TM == 1 only): the wave carries two box rows; operand/accumulator slot u (the "tile"
// index) is the box, both use output tile 0 of W.  PG > 1 (packed, PAIR only): slot u is a group
// of PG boxes sharing the tile (block-diagonal weights); layer 0 builds its identity-form
// operands on the fly from the boxes' input ranges in the wave's LDS box table.
template <int NT, int TM, bool PAIR, int PG = 1, class S = SymShapeAny>
__device__ __forceinline__ void fa_sym_layer(const NetDesc& net, const BoundArgs& a, const SymCfg& cfg,
                                             const float* smem, float* T, const float* bxv, const int* cdim_s,
                                             int l, int r, int node, int r2, int node2, bool v2, int lane,
                                             const float (&B)[NT][PAIR ? 2 : TM][2][4],
                                             float (&A)[NT][PAIR ? 2 : TM][2][4]) {
  constexpr int TMS = PAIR ? 2 : TM;
  constexpr bool CR = SymForm<PAIR, TM>::CR;
  constexpr int TS = SymSlab<NT>::TS;
  constexpr bool CS = S::L > 0;        // compile-time shape: l is a constant here (fa_sym_layers_c)
  const int col = lane & 15, grp = lane >> 4;
  const int n_in = CS ? S::dim(l) : net.dims[l], n_out = CS ? S::dim(l + 1) : net.dims[l + 1];
  const int tin = (n_in + 15) >> 4, tout = (n_out + 15) >> 4;
  const float* sw = smem + cfg.w_lds[l];
  const float* sb = smem + cfg.b_lds[l];
  const bool last = CS ? l == S::L - 1 : l == net.n_layers - 1;
  const float gg = net.g_gemm[l];
  const float gc = net.g_conc;
  const float gi = net.g_one;
  const float unit = net.unit;
  const float gnext = last ? 0.f : net.g_gemm[l + 1];
  const int noff = net.neuron_off[l];
  const int nc = cfg.nc;
  const int n0 = net.dims[0];
  // neuron lane role in the epilogue: lanes 0-15 = U block, 16-31 = L block of neuron (lane & 15)
  const bool nl_act = lane < 32;
  const int ob = (lane >> 4) & 1;
#ifndef FA_SYM_TIMING_NO_EPILOGUE
  if (PG > 1 && l == 0) {
    // packed layer 0: group u accumulates its PG boxes, box g through tile g of the packed W_0
    // (W_0 placed at output rows g * 16 / PG ..), K = the box's own input dims
    const float* boxtab = bxv + 2 * PG * SymSlab<NT, PG>::BOX;   // [2 PG][lo 16 | hi 16]
    const float g0 = net.g_gemm[0];
    const int n0v = net.dims[0];
    f32x4 U[2][NT], Lq[2][NT];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) U[u][ct] = Lq[u][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int g = 0; g < PG; ++g) {
        const float* bt = boxtab + (u * PG + g) * 32;
        const float4 w4 = reinterpret_cast<const float4*>(sw)[g * 64 + lane];
        const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = 4 * grp + i;
          const bool kv = k < n0v;
          const float xl = kv ? bt[k] : 0.f, xh = kv ? bt[16 + k] : 0.f;
          const bool folded = kv && ((cfg.fold >> k) & 1ull);
          const float m = fmaxf(fabsf(xl), fabsf(xh));
          const float wp = fmaxf(wv[i], 0.f), wn = fminf(wv[i], 0.f);
#pragma unroll
          for (int ct = 0; ct < NT; ++ct) {
            const int c = ct * 16 + col;
            float vu = 0.f, vl = 0.f;
            if (kv) {
              if (c >= 4) {
                vu = vl = (!folded && c - 4 < nc && cdim_s[c - 4] == k) ? 1.f : 0.f;
              } else if (c == 0) {
                vu = vl = folded ? xl : 0.f;
              } else if (c == 1) {
                vu = g0 * m; vl = -vu;
              } else if (c == 2) {
                vu = xh; vl = xl;
              } else {
                vu = g0 * fabsf(xh); vl = -(g0 * fabsf(xl));
              }
            }
            U[u][ct] = fa_mfma4(wp, vu, U[u][ct]);
            Lq[u][ct] = fa_mfma4(wp, vl, Lq[u][ct]);
            U[u][ct] = fa_mfma4(wn, vl, U[u][ct]);
            Lq[u][ct] = fa_mfma4(wn, vu, Lq[u][ct]);
          }
        }
      }
    }
    float nu[2][NT][4], nlo[2][NT][4];
    if (!fa_sym_epilogue<NT, PAIR, PG, CR, S>(net, a, cfg, smem, T, bxv, cdim_s, l, r, node, r2, node2, v2, lane, 0, U, Lq,
                                       nu, nlo))
      return;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          A[ct][u][0][i] = nu[u][ct][i];
          A[ct][u][1][i] = nlo[u][ct][i];
        }
    return;
  }
  if (PG == 1 && last && n_out == 1) {
    // single-neuron output layer: a VALU dot product instead of a 16-row MFMA tile of which
    // 15 rows are padding.  Lane (grp, col) sums its 4*tin neurons k = 16t + 4 grp + i for its
    // form column; two cross-group butterflies finish the sum (any summation order stays within
    // the layer's gamma_{2 n_in + 1} bound).  W[k][0] is lane (grp*16) of the permuted block.
    constexpr int NB = PAIR ? 2 : 1;   // boxes carried by the wave
    float su[NB][NT], sl[NB][NT];
#pragma unroll
    for (int bi = 0; bi < NB; ++bi)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) su[bi][ct] = sl[bi][ct] = 0.f;
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      if (t >= tin) break;
      const float4 w4 = reinterpret_cast<const float4*>(sw)[t * 64 + grp * 16];
      const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float wp = fmaxf(wv[i], 0.f), wn = fminf(wv[i], 0.f);
#pragma unroll
        for (int bi = 0; bi < NB; ++bi)
#pragma unroll
          for (int ct = 0; ct < NT; ++ct) {
            const int bt = PAIR ? bi : t;
            if (CR) {   // su = W C, sl = |W| R
              su[bi][ct] = fmaf(wv[i], B[ct][bt][0][i], su[bi][ct]);
              sl[bi][ct] = fmaf(fabsf(wv[i]), B[ct][bt][1][i], sl[bi][ct]);
            } else {
              su[bi][ct] = fmaf(wp, B[ct][bt][0][i], fmaf(wn, B[ct][bt][1][i], su[bi][ct]));
              sl[bi][ct] = fmaf(wp, B[ct][bt][1][i], fmaf(wn, B[ct][bt][0][i], sl[bi][ct]));
            }
          }
      }
    }
    f32x4 U[2][NT], Lq[2][NT];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) U[1][ct] = Lq[1][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int bi = 0; bi < NB; ++bi)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) {
        float xu = su[bi][ct], xl = sl[bi][ct];
        xu += __shfl_xor(xu, 16, 64);
        xl += __shfl_xor(xl, 16, 64);
        xu += __shfl_xor(xu, 32, 64);
        xl += __shfl_xor(xl, 32, 64);
        U[bi][ct] = f32x4{grp == 0 ? xu : 0.f, 0.f, 0.f, 0.f};     // row 0 of tile bi = neuron 0
        Lq[bi][ct] = f32x4{grp == 0 ? xl : 0.f, 0.f, 0.f, 0.f};
        if (CR) fa_pq_to_ul(f32x4(U[bi][ct]), f32x4(Lq[bi][ct]), ct * 16 + col, gg, U[bi][ct], Lq[bi][ct]);
      }
    float nu[2][NT][4], nlo[2][NT][4];
    fa_sym_epilogue<NT, PAIR, PG, CR, S>(net, a, cfg, smem, T, bxv, cdim_s, l, r, node, r2, node2, v2, lane, 0, U, Lq,
                                  nu, nlo);
    return;
  }
#endif
#pragma unroll
  for (int jt0 = 0; jt0 < TM; jt0 += 2) {
    if (jt0 >= tout) break;
    f32x4 U[2][NT], Lq[2][NT];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int jt = jt0 + u;
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) {
        U[u][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
        Lq[u][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      if (PAIR ? (jt0 > 0) : (jt >= tout || jt >= TM)) continue;
      const float4* wq = reinterpret_cast<const float4*>(sw) + (size_t)(PAIR ? 0 : jt) * tin * 64 + lane;
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        if (t >= tin) break;
        const float4 w4 = wq[t * 64];
        const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float wp = fmaxf(wv[i], 0.f), wn = fminf(wv[i], 0.f);
#pragma unroll
          for (int ct = 0; ct < NT; ++ct) {
            const int bt = PAIR ? u : t;
            const float bu = B[ct][bt][0][i], bl = B[ct][bt][1][i];
            if (CR) {   // U = P = W C, Lq = Q = |W| R
              U[u][ct] = fa_mfma4(wv[i], bu, U[u][ct]);
              Lq[u][ct] = fa_mfma4(fabsf(wv[i]), bl, Lq[u][ct]);
            } else {
              U[u][ct] = fa_mfma4(wp, bu, U[u][ct]);
              Lq[u][ct] = fa_mfma4(wp, bl, Lq[u][ct]);
              U[u][ct] = fa_mfma4(wn, bl, U[u][ct]);
              Lq[u][ct] = fa_mfma4(wn, bu, Lq[u][ct]);
            }
          }
        }
      }
      if (CR) {
#pragma unroll
        for (int ct = 0; ct < NT; ++ct)
          fa_pq_to_ul(f32x4(U[u][ct]), f32x4(Lq[u][ct]), ct * 16 + col, gg, U[u][ct], Lq[u][ct]);
      }
    }
    float nu[2][NT][4], nlo[2][NT][4];
#ifdef FA_SYM_TIMING_NO_EPILOGUE
    // timing-only build (tools/symk_timing.cpp): GEMM + operand hand-off without the epilogue
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          nu[u][ct][i] = U[u][ct][i] * 1e-3f;
          nlo[u][ct][i] = Lq[u][ct][i] * 1e-3f;
        }
    if (l == net.n_layers - 1) {
      if (lane == 0) a.out_lb[r] = nu[0][0][0] + nlo[0][0][1];
      continue;
    }
#else
    if (!fa_sym_epilogue<NT, PAIR, PG, CR, S>(net, a, cfg, smem, T, bxv, cdim_s, l, r, node, r2, node2, v2, lane, jt0, U,
                                       Lq, nu, nlo))
      continue;
#endif
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (jt0 + u >= TMS) break;
#pragma unroll
      for (int ct = 0; ct < NT; ++ct)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          A[ct][jt0 + u][0][i] = nu[u][ct][i];
          A[ct][jt0 + u][1][i] = nlo[u][ct][i];
        }
    }
  }
}

// Minimum waves per SIMD the register allocator must leave room for (VGPR budget 512 / waves):
// the paired single-tile kernel needed 180 VGPRs (2 waves/SIMD) and the 4-tile kernel 260 (1 wave),
// both spill-free at 3 / 2 waves (167 / 242 VGPRs).  The 7-tile kernel (366 VGPRs, its operand
// ping-pong alone is 112) at 2 waves spills 284 B/lane to scratch and still wins where LDS allows
// a second block: AC-2 1.56 -> 0.99 ms per 131 072 rows; AC-4 (63 KB of staged W) is LDS-bound
// at one block per CU, so its workgroups carry 8 waves (FA_SYM_BIG_THREADS): 3.98 -> 2.89 ms.  The
// 4-tile kernel at 3 waves (244 B/lane scratch): AC-5 1.297 -> 1.237, AC-7 1.363 -> 1.292 ms
// (tools/ab_micro.sh, profiles/r2/s3/).
#ifndef FA_SYM_WPE7
#define FA_SYM_WPE7 2
#endif
#ifndef FA_SYM_WPE4
#define FA_SYM_WPE4 2   // round 3: 2 waves/SIMD beat 3 (1157 vs 1174 ms/step, 3 alternating runs each,
                        // profiles/r3/ab/wpe4.md)
#endif
#define FA_SYM_WAVES_PER_EU(NT, TM, PAIR) \
  ((PAIR) ? 3 : ((TM) == 2 ? 3 : ((TM) == 4 ? FA_SYM_WPE4 : ((TM) == 7 ? FA_SYM_WPE7 : 1))))

// The layer chain of a compile-time shape: one inlined fa_sym_layer per layer, l a constant in each,
// operands ping-ponging between XA (even layers' input) and XB.
template <int NT, int TM, bool PAIR, int PG, class S, int... LS>
__device__ __forceinline__ void fa_sym_layers_c(std::integer_sequence<int, LS...>, const NetDesc& net,
                                                const BoundArgs& a, const SymCfg& cfg, const float* smem, float* T,
                                                const float* bxv, const int* cdim_s, int r, int node, int r2,
                                                int node2, bool v2, int lane, float (&XA)[NT][PAIR ? 2 : TM][2][4],
                                                float (&XB)[NT][PAIR ? 2 : TM][2][4]) {
  ((LS & 1 ? fa_sym_layer<NT, TM, PAIR, PG, S>(net, a, cfg, smem, T, bxv, cdim_s, LS, r, node, r2, node2, v2, lane,
                                               XB, XA)
           : fa_sym_layer<NT, TM, PAIR, PG, S>(net, a, cfg, smem, T, bxv, cdim_s, LS, r, node, r2, node2, v2, lane,
                                               XA, XB)),
   ...);
}

// Threads per workgroup: the 7-tile kernel's staged W (AC-4: 63 KB) leaves LDS for one workgroup
// per CU, so it runs 8 waves per workgroup (2 per SIMD, its VGPR limit) instead of 4.
#ifndef FA_SYM_BIG_THREADS
#define FA_SYM_BIG_THREADS 512
#endif
#define FA_SYM_THREADS(TM) ((TM) == 7 ? FA_SYM_BIG_THREADS : FA_THREADS)

template <int NT, int TM, bool PAIR, int PG = 1, class S = SymShapeAny>
__global__ void __launch_bounds__(FA_SYM_THREADS(TM)) __attribute__((amdgpu_waves_per_eu(FA_SYM_WAVES_PER_EU(NT, TM, PAIR))))
fa_sym_kernel(NetDesc net, BoundArgs a, SymCfg cfg) {
  constexpr bool CR = SymForm<PAIR, TM>::CR;   // centre / radius operands (multi-tile kernels)
  constexpr int TMS = PAIR ? 2 : TM;   // operand slots: K tiles, or (PAIR) the wave's two boxes /
                                       // (packed) two groups of PG boxes
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  // ---- stage the MFMA-operand-order weights + biases (pre-permuted in `flat`; the block-diagonal
  //      packed copy when PG > 1) into LDS
  {
    const float4* src = reinterpret_cast<const float4*>(a.flat + cfg.stage_off);
    float4* dst = reinterpret_cast<float4*>(smem);
    for (int e = tid; e < (cfg.stage_floats >> 2); e += FA_SYM_THREADS(TM)) dst[e] = src[e];
  }
  int* cdim_s = reinterpret_cast<int*>(smem + cfg.lds_floats - FA_SYM_MAXC);
  for (int c = tid; c < FA_SYM_MAXC; c += FA_SYM_THREADS(TM)) cdim_s[c] = c < cfg.nc ? cfg.cdim[c] : -1;
  __syncthreads();
  const int lane = tid & 63;
  const int grp = lane >> 4;
  const int wave = tid >> 6;
  const int nw = FA_SYM_THREADS(TM) / 64;
  const int n0 = S::L > 0 ? S::dim(0) : net.dims[0];
  const int nc = cfg.nc;
  const float g0 = net.g_gemm[0];
  float* T = smem + cfg.lds_floats + wave * SymSlab<NT, PG>::FLOATS;
  float* bxv = T + SymSlab<NT>::TILE;             // [lo | hi | max(|lo|,|hi|)] per coefficient column
  const int tin0 = (n0 + 15) >> 4;
  // column layout: 0 constant, 1 error, 2 interval, 3 interval error, 4.. coefficients
  int role[NT], cdm[NT];
#pragma unroll
  for (int ct = 0; ct < NT; ++ct) {
    const int c = ct * 16 + (lane & 15);
    role[ct] = c == 0 ? 1 : c == 1 ? 2 : c == 2 ? 3 : c == 3 ? 4 : (c - 4 < nc ? 0 : 5);
    cdm[ct] = (role[ct] == 0) ? cdim_s[c - 4] : -1;
  }
  constexpr int RPW = PAIR ? 2 * PG : 1;   // box rows per wave and pass
  for (int r0 = (blockIdx.x * nw + wave) * RPW; r0 < a.R; r0 += gridDim.x * nw * RPW) {
    const int r = __builtin_amdgcn_readfirstlane(r0);
    const bool v2 = PAIR && r + 1 < a.R;           // second row valid (else it shadows r, no writes)
    const int rb = v2 ? r + 1 : r;
    if (a.skip_status) {   // BaB: rows of partitions already decided / stopped are not bounded
      bool any = false;
#pragma unroll
      for (int bi = 0; bi < RPW; ++bi) {
        const int rr = min(r + bi, a.R - 1);
        const int8_t s1 = a.skip_status[a.skip_part[a.V > 0 ? rr / a.V : rr]];
        any = any || s1 == 3 || s1 == 4;
      }
      if (!any) continue;   // wave-uniform (r is)
    }
    SymBox bxs[RPW];
#pragma unroll
    for (int bi = 0; bi < RPW; ++bi) {
      SymBox& bx = bxs[bi];
      const int rr = PG > 1 ? min(r + bi, a.R - 1) : (bi ? rb : r);
      bx.a = &a;
      bx.n0 = n0;
      bx.node = a.V > 0 ? rr / a.V : rr;
      bx.v = a.V > 0 ? rr - bx.node * a.V : 0;
      if (lane < FA_SYM_MAXC) {   // box values per column (0 on non-coefficient columns)
        float* bv = bxv + bi * SymSlab<NT>::BOX;
        const int d = (lane >= 4 && lane - 4 < nc) ? cdim_s[lane - 4] : -1;
        const float l0 = d >= 0 ? bx.lo(d) : 0.f, h0 = d >= 0 ? bx.hi(d) : 0.f;
        // centre / radius / magnitude of the column's range: exact for lattice boxes (integers
        // below 2^22); any other range is enclosed outward ([mid - rad, mid + rad] contains it and
        // m >= |mid| + rad), which keeps every bound sound
        float mid = 0.5f * (l0 + h0), rad = 0.5f * (h0 - l0), mm = fmaxf(fabsf(l0), fabsf(h0));
        const bool lattice = l0 == rintf(l0) && h0 == rintf(h0) && fabsf(l0) < 4194304.f && fabsf(h0) < 4194304.f;
        if (!lattice) {
          rad = nextafterf(fmaxf(h0 - mid, mid - l0), INFINITY);
          mm = nextafterf(fabsf(mid) + rad, INFINITY);
        }
        bv[lane] = mid;
        bv[FA_SYM_MAXC + lane] = rad;
        bv[2 * FA_SYM_MAXC + lane] = mm;
      }
      if (PG > 1 && lane < 32) {   // packed: the box's input ranges for the layer-0 operands
        const int d = lane & 15;
        float* bt = bxv + 2 * PG * SymSlab<NT, PG>::BOX + bi * 32;
        bt[lane] = d < n0 ? (lane < 16 ? bx.lo(d) : bx.hi(d)) : 0.f;
      }
    }
    const SymBox& bx = bxs[0];
    float XA[NT][TMS][2][4], XB[NT][TMS][2][4];
    // ---- layer-0 operands: identity forms (folded dims -> constant) + [hi | lo] interval rows;
    //      L-block error columns negated
#pragma unroll
    for (int t = 0; t < TMS; ++t) {
      if (PG > 1) break;                      // packed: layer-0 operands built on the fly
      if (!PAIR && t >= tin0) break;
      const SymBox& bt = bxs[PAIR ? t : 0];   // PAIR: slot t = box t (n0 <= 16: one K tile)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = (PAIR ? 0 : 16 * t) + 4 * grp + i;
        float xl = 0.f, xh = 0.f;
        const bool kv = k < n0;
        if (kv) {
          xl = bt.lo(k);
          xh = bt.hi(k);
        }
        const bool folded = kv && ((cfg.fold >> k) & 1ull);
        const float m = fmaxf(fabsf(xl), fabsf(xh));
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) {
          float vu = 0.f, vl = 0.f;
          if (kv) {
            switch (role[ct]) {
              // C/R kernels: (vu, vl) hold the centre / radius of the [upper | lower] operand pair
              case 0: vu = (!folded && cdm[ct] == k) ? 1.f : 0.f; vl = CR ? 0.f : vu; break;
              case 1: vu = folded ? xl : 0.f; vl = CR ? 0.f : vu; break;
              case 2: vu = CR ? 0.f : g0 * m; vl = CR ? g0 * m : -vu; break;
              case 3:
                vu = CR ? 0.5f * (xh + xl) : xh;
                vl = CR ? 0.5f * (xh - xl) : xl;
                break;
              case 4:
                vu = CR ? 0.5f * g0 * (fabsf(xh) - fabsf(xl)) : g0 * fabsf(xh);
                vl = CR ? 0.5f * g0 * (fabsf(xh) + fabsf(xl)) : -(g0 * fabsf(xl));
                break;
              default: break;
            }
          }
          XA[ct][t][0][i] = vu;
          XA[ct][t][1][i] = vl;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    if constexpr (S::L > 0) {
      fa_sym_layers_c<NT, TM, PAIR, PG, S>(std::make_integer_sequence<int, S::L>{}, net, a, cfg, smem, T, bxv, cdim_s,
                                           r, bx.node, rb, bxs[RPW - 1].node, v2, lane, XA, XB);
    } else {
      for (int l = 0; l < net.n_layers; ++l) {
        if (l & 1)
          fa_sym_layer<NT, TM, PAIR, PG>(net, a, cfg, smem, T, bxv, cdim_s, l, r, bx.node, rb, bxs[RPW - 1].node, v2,
                                         lane, XB, XA);
        else
          fa_sym_layer<NT, TM, PAIR, PG>(net, a, cfg, smem, T, bxv, cdim_s, l, r, bx.node, rb, bxs[RPW - 1].node, v2,
                                         lane, XA, XB);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// (A K-split variant with two waves per box -- each wave holding half of the K tiles and
// exchanging partial sums through LDS, two workgroup barriers per layer -- reached 2 waves/SIMD
// for the 100-wide layers but measured 10-75 % SLOWER than one wave per box on every AC shape:
// profiles/experiments/r1_bounds_microbench_ksplit_2waves_per_box.json.  Not kept.)

namespace {

typedef void (*SymKernel)(NetDesc, BoundArgs, SymCfg);

template <int NT, int TM, bool PAIR = false, int PG = 1>
SymKernel sym_ptr() {
  return fa_sym_kernel<NT, TM, PAIR, PG>;
}

// several boxes per MFMA tile for narrow networks (FAIRIFY_SYM_PACK=0 turns it off for A/B runs)
bool use_pack() {
  static const bool v = [] {
    const char* e = getenv("FAIRIFY_SYM_PACK");
    return !(e && *e == '0');
  }();
  return v;
}

SymKernel select_packed(int pg) {
  switch (pg) {
    case 2: return sym_ptr<1, 1, true, 2>();
    case 4: return sym_ptr<1, 1, true, 4>();
    default: return nullptr;
  }
}

// two box rows per wave for single-tile networks (FAIRIFY_SYM_PAIR=0 turns it off for A/B runs)
bool use_pair() {
  static const bool v = [] {
    const char* e = getenv("FAIRIFY_SYM_PAIR");
    return !(e && *e == '0');
  }();
  return v;
}

// widest layer (in 16-neuron tiles) served by the register-resident kernel; FAIRIFY_SYM_MAX_TM
// lowers it for A/B runs against the LDS-tiled kernel
int max_tm() {
  static const int v = [] {
    const char* e = getenv("FAIRIFY_SYM_MAX_TM");
    return (e && *e) ? atoi(e) : 10;
  }();
  return v;
}

SymKernel select_kernel(int NT, int TM) {
  if (TM > max_tm()) return nullptr;
  switch (NT) {
    case 1:
      if (TM <= 1) return use_pair() ? sym_ptr<1, 1, true>() : sym_ptr<1, 1>();
      if (TM <= 2) return sym_ptr<1, 2>();
      if (TM <= 4) return sym_ptr<1, 4>();
      if (TM <= 7) return sym_ptr<1, 7>();
      if (TM <= 10) return sym_ptr<1, 10>();   // e.g. BM-4's 150-wide layer (scratch-backed operands)
      return nullptr;
    case 2:
      if (TM <= 1) return sym_ptr<2, 1>();
      if (TM <= 2) return sym_ptr<2, 2>();
      if (TM <= 4) return sym_ptr<2, 4>();
      if (TM <= 10) return sym_ptr<2, 10>();
      return nullptr;
    case 3:
      if (TM <= 1) return sym_ptr<3, 1>();
      if (TM <= 2) return sym_ptr<3, 2>();
      return nullptr;
    default:
      return nullptr;
  }
}

// the TM template bucket select_kernel uses for a layer width of TM tiles (0: none)
int tm_bucket(int NT, int TM) {
  if (TM > max_tm()) return 0;
  const int b = TM <= 1 ? 1 : TM <= 2 ? 2 : TM <= 4 ? 4 : TM <= 7 ? 7 : TM <= 10 ? 10 : 0;
  if (NT == 2 && b == 7) return 10;
  if (NT == 3 && b > 2) return 0;
  return NT >= 1 && NT <= 3 ? b : 0;
}

// Compile-time shapes (SymShape): the zoo's dominant layer chains, each instantiated for the (NT, TM
// bucket) kernel the run-time selection picks for it, so launch geometry, LDS layout and arithmetic
// are the generic kernel's.  FAIRIFY_SYM_SHAPED=0 (read per launch: the bitwise-equality test
// toggles it) keeps the run-time-shape kernels.
struct ShapedKernel {
  int nt, tm;
  std::vector<int> dims;
  SymKernel k;
};
template <int NT, int TM, int... D>
ShapedKernel shaped() {
  return {NT, TM, {D...}, fa_sym_kernel<NT, TM, false, 1, SymShape<D...>>};
}

const std::vector<ShapedKernel>& shaped_kernels() {
  static const std::vector<ShapedKernel> v = {
      shaped<1, 4, 13, 64, 32, 16, 8, 4, 1>(),   // AC-7, PA folded (node-row expansion)
      shaped<2, 4, 13, 64, 32, 16, 8, 4, 1>(),   // AC-7, no dim folded (beta tightening rows)
      shaped<2, 4, 16, 64, 32, 16, 8, 4, 1>(),   // BM-8
      shaped<1, 4, 13, 64, 64, 1>(),             // AC-5
      shaped<1, 4, 13, 50, 1>(),                 // AC-3
      shaped<1, 7, 13, 100, 100, 1>(),           // AC-4
      shaped<1, 7, 13, 100, 1>(),                // AC-2
  };
  return v;
}

SymKernel select_shaped(const NetDesc& net, int NT, int tmb) {
  const char* e = getenv("FAIRIFY_SYM_SHAPED");
  if (e && *e == '0') return nullptr;
  for (const auto& s : shaped_kernels()) {
    if (s.nt != NT || s.tm != tmb || (int)s.dims.size() != net.n_layers + 1) continue;
    bool same = true;
    for (int l = 0; l <= net.n_layers && same; ++l) same = s.dims[l] == net.dims[l];
    if (same) return s.k;
  }
  return nullptr;
}

int device_cus() {
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

// Launch the register-resident kernel if the shape fits; returns 1 if launched, 0 if the caller
// must use the LDS-tiled kernel, <0 on a launch error.  fold_mask: input dims degenerate in
// every row (PA dims under node-row expansion).
extern "C" int fa_sym_try_launch(const NetDesc& net, BoundArgs a, unsigned long long fold_mask,
                                 hipStream_t stream) {
  if (!a.symbolic || a.R <= 0) return 0;
  const int n0 = net.dims[0];
  if (n0 > 64) return 0;
  SymCfg cfg{};
  cfg.fold = fold_mask;
  int nc = 0;
  for (int d = 0; d < n0; ++d)
    if (!((fold_mask >> d) & 1ull)) {
      if (nc >= FA_SYM_MAXC) return 0;
      cfg.cdim[nc++] = d;
    }
  cfg.nc = nc;
  const int cols = nc + 4;
  const int NT = (cols + 15) / 16;
  int TM = 1;
  for (int l = 0; l < net.n_layers; ++l) TM = std::max(TM, (net.dims[l] + 15) / 16);
  TM = std::max(TM, (net.dims[net.n_layers] + 15) / 16);
  SymKernel k = select_kernel(NT, TM);
  if (!k) return 0;
  const bool pair0 = k == sym_ptr<1, 1, true>();
  const int tmb = tm_bucket(NT, TM);
  // packed narrow networks: pack_g boxes per tile, block-diagonal weights (NetDesc.pack_*)
  const int pg = (pair0 && net.pack_g > 1 && net.dims[0] <= 16 && use_pack()) ? net.pack_g : 1;
  if (pg > 1) k = select_packed(pg);
  if (!k) return 0;
  if (!pair0) {   // a compile-time-shape instance of the same (NT, TM) kernel, when there is one
    const SymKernel ks = select_shaped(net, NT, tmb);
    if (ks) k = ks;
  }
  int off = 0;
  if (pg > 1) {
    cfg.w_lds[0] = 0;
    off = pg * 256;
    for (int l = 1; l < net.n_layers; ++l) {
      cfg.w_lds[l] = off;
      off += 256;
    }
    for (int l = 0; l < net.n_layers; ++l) {
      cfg.b_lds[l] = off;
      off += 16;
    }
    if (off != net.pack_floats) return -1;      // layout mismatch with the packed block
    cfg.stage_off = net.pack_off;
  } else {
    for (int l = 0; l < net.n_layers; ++l) {
      cfg.w_lds[l] = off;
      off += ((net.dims[l] + 15) / 16) * ((net.dims[l + 1] + 15) / 16) * 256;
    }
    for (int l = 0; l < net.n_layers; ++l) {
      cfg.b_lds[l] = off;
      off += net.dims[l + 1];
    }
    off = ((off + 3) & ~3);
    if (off != net.wperm_floats) return -1;       // layout mismatch with the pre-permuted block
    cfg.stage_off = net.wperm_off;
  }
  cfg.stage_floats = off;
  off += FA_SYM_MAXC;                           // + column -> input-dim table (ints)
  cfg.lds_floats = off;
  int slab = 0;
  switch (NT) {
    case 1:
      slab = pg == 2 ? SymSlab<1, 2>::FLOATS : pg == 4 ? SymSlab<1, 4>::FLOATS : SymSlab<1>::FLOATS;
      break;
    case 2: slab = SymSlab<2>::FLOATS; break;
    default: slab = SymSlab<3>::FLOATS; break;
  }
  const int threads = (!pair0 && NT == 1 && tmb == 7) ? FA_SYM_BIG_THREADS : FA_THREADS;   // = FA_SYM_THREADS(TM)
  const int rows_per_block = (threads / 64) * (pair0 ? 2 * pg : 1);
  const size_t bytes = (size_t)(off + (threads / 64) * slab) * sizeof(float);
  if (bytes > 160 * 1024) return 0;
  // per (kernel, LDS bytes): raise the dynamic-LDS limit once and cache the occupancy
  static std::mutex mu;
  static std::map<std::pair<const void*, size_t>, int> occ;
  int per_cu = 0;
  {
    std::lock_guard<std::mutex> g(mu);
    const auto key = std::make_pair((const void*)k, bytes);
    auto it = occ.find(key);
    if (it == occ.end()) {
      if (!fa_lds_ok(bytes)) return -4;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, threads, bytes) != hipSuccess || per_cu <= 0)
        per_cu = 1;
      occ[key] = per_cu;
    } else {
      per_cu = it->second;
    }
  }
  long long blocks = (a.R + rows_per_block - 1) / rows_per_block;
  const long long cap = (long long)device_cus() * per_cu;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(threads), bytes, stream, net, a, cfg);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 1 : -(int)e;
}

FA_LDS_REGISTER(FA_LDS_K((sym_ptr<1, 1>())), FA_LDS_K((sym_ptr<1, 1, true>())), FA_LDS_K((sym_ptr<1, 1, true, 2>())),
                FA_LDS_K((sym_ptr<1, 1, true, 4>())), FA_LDS_K((sym_ptr<1, 2>())), FA_LDS_K((sym_ptr<1, 4>())),
                FA_LDS_K((sym_ptr<1, 7>())), FA_LDS_K((sym_ptr<1, 10>())), FA_LDS_K((sym_ptr<2, 1>())),
                FA_LDS_K((sym_ptr<2, 2>())), FA_LDS_K((sym_ptr<2, 4>())), FA_LDS_K((sym_ptr<2, 10>())),
                FA_LDS_K((sym_ptr<3, 1>())), FA_LDS_K((sym_ptr<3, 2>())));
FA_LDS_REGISTER(FA_LDS_K((fa_sym_kernel<1, 4, false, 1, SymShape<13, 64, 32, 16, 8, 4, 1>>)),
                FA_LDS_K((fa_sym_kernel<2, 4, false, 1, SymShape<13, 64, 32, 16, 8, 4, 1>>)),
                FA_LDS_K((fa_sym_kernel<2, 4, false, 1, SymShape<16, 64, 32, 16, 8, 4, 1>>)),
                FA_LDS_K((fa_sym_kernel<1, 4, false, 1, SymShape<13, 64, 64, 1>>)),
                FA_LDS_K((fa_sym_kernel<1, 4, false, 1, SymShape<13, 50, 1>>)),
                FA_LDS_K((fa_sym_kernel<1, 7, false, 1, SymShape<13, 100, 100, 1>>)),
                FA_LDS_K((fa_sym_kernel<1, 7, false, 1, SymShape<13, 100, 1>>)));
