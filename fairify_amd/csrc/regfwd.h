// Register-resident concrete forward of 16 points per wave64 (gfx950 MFMA), W from LDS.
//
// Same layout as the rigorous point kernel (csrc/points.hip) without the error term: the 16
// points are the 16 columns of v_mfma_f32_16x16x4_f32 tiles whose rows are neurons, so layer
// l's accumulator tile is directly layer l+1's B operand (register i of tile t = neuron
// 16t + 4*(lane>>4) + i of point lane&15) and activations never touch LDS or HBM.  W comes from
// the MFMA-operand-order block of `flat` (ops/backend.py:mfma_weight_block) staged in LDS: one
// 16-byte ds_read per lane per 4 MFMAs.
#pragma once
#include "args.h"

// LDS float offsets of each layer's permuted W and bias inside the staged block.
struct RegNetCfg {
  int w_lds[FA_MAX_LAYERS];
  int b_lds[FA_MAX_LAYERS];
  int floats;                 // staged block size (== net.wperm_floats)
};

// Host helper: offsets of the permuted block; returns false on a layout mismatch.
inline bool fa_regnet_cfg(const NetDesc& net, RegNetCfg& cfg) {
  int off = 0;
  for (int l = 0; l < net.n_layers; ++l) {
    cfg.w_lds[l] = off;
    off += ((net.dims[l] + 15) / 16) * ((net.dims[l + 1] + 15) / 16) * 256;
  }
  for (int l = 0; l < net.n_layers; ++l) {
    cfg.b_lds[l] = off;
    off += net.dims[l + 1];
  }
  cfg.floats = (off + 3) & ~3;
  return cfg.floats == net.wperm_floats;
}

// Largest 16-neuron tile count over all layers (input included): the register tile depth.
inline int fa_regnet_tm(const NetDesc& net) {
  int tm = 1;
  for (int l = 0; l <= net.n_layers; ++l) tm = tm > (net.dims[l] + 15) / 16 ? tm : (net.dims[l] + 15) / 16;
  return tm;
}

// Stage the permuted W + biases (flat + wperm_off) into LDS with float4 copies (all threads).
__device__ __forceinline__ void fa_stage_wperm(const NetDesc& net, const float* flat, float* smem, int tid,
                                               int nthreads) {
  const float4* src = reinterpret_cast<const float4*>(flat + net.wperm_off);
  float4* dst = reinterpret_cast<float4*>(smem);
  for (int e = tid; e < (net.wperm_floats >> 2); e += nthreads) dst[e] = src[e];
}

// One layer: H (inputs of layer l) -> H2 (ReLU outputs; padded neurons 0).  On the last layer
// returns the logit of point lane&15 in lanes 0..15 (other lanes: unspecified).
// ``dead`` (optional, LDS or global): per hidden neuron (all-neuron numbering) forced-zero flags.
template <int TM>
__device__ __forceinline__ float fa_reg_layer(const NetDesc& net, const RegNetCfg& cfg, const float* sw_all, int l,
                                              int lane, const float (&H)[TM][4], float (&H2)[TM][4],
                                              const uint8_t* dead = nullptr) {
  const int grp = lane >> 4;
  const int n_in = net.dims[l], n_out = net.dims[l + 1];
  const int tin = (n_in + 15) >> 4, tout = (n_out + 15) >> 4;
  const float4* sw = reinterpret_cast<const float4*>(sw_all + cfg.w_lds[l]);
  const float* sb = sw_all + cfg.b_lds[l];
  const bool last = l == net.n_layers - 1;
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
      if (jt == 0) logit = Z[0] + sb[0];
      continue;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = 16 * jt + 4 * grp + i;
      const bool zero = j >= n_out || (dead && dead[net.neuron_off[l] + j]);
      H2[jt][i] = zero ? 0.f : fmaxf(Z[i] + sb[j], 0.f);
    }
  }
  return logit;
}

// Full forward of the 16 points held in HA (layer-0 layout: HA[t][i] = x_col[16t + 4 grp + i],
// zero beyond n0).  HA and HB are clobbered.  Logit of point lane&15 in lanes 0..15.
template <int TM>
__device__ __forceinline__ float fa_reg_forward(const NetDesc& net, const RegNetCfg& cfg, const float* sw_all,
                                                int lane, float (&HA)[TM][4], float (&HB)[TM][4],
                                                const uint8_t* dead = nullptr) {
  float z = 0.f;
  for (int l = 0; l < net.n_layers; ++l) {
    if (l & 1) z = fa_reg_layer<TM>(net, cfg, sw_all, l, lane, HB, HA, dead);
    else z = fa_reg_layer<TM>(net, cfg, sw_all, l, lane, HA, HB, dead);
  }
  return z;
}
