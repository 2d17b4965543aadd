// Standalone timing of the register-resident symbolic kernel on an AC-4-shaped net
// (13 -> 100 -> 100 -> 1, PA folded), with and without the epilogue
// (build twice: hipcc ... [-DFA_SYM_TIMING_NO_EPILOGUE]).  Random weights and boxes.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "../fairify_amd/csrc/args.h"

extern "C" int fa_sym_try_launch(const NetDesc& net, BoundArgs a, unsigned long long fold_mask, hipStream_t st);

static float gamma_up(int k, double u) { double ku = (k + 2) * u; return std::nextafter((float)(ku / (1 - ku)), INFINITY); }

int main(int argc, char** argv) {
  std::vector<int> dims = {13, 100, 100, 1};
  const int R = argc > 1 ? atoi(argv[1]) : 65536;
  NetDesc d{};
  d.n_layers = 3;
  int off = 0, noff = 0;
  for (int i = 0; i < 4; ++i) d.dims[i] = dims[i];
  for (int l = 0; l < 3; ++l) {
    d.w_off[l] = off; off += dims[l] * dims[l + 1];
    d.b_off[l] = off; off += dims[l + 1];
    d.neuron_off[l] = noff; noff += dims[l + 1];
    d.g_gemm[l] = gamma_up(2 * dims[l] + 1, 1.0 / (1 << 24));
    d.g_fwd[l] = gamma_up(dims[l] + 1, 1.0 / (1 << 24));
  }
  d.n_neurons = noff; d.n_hidden = noff - 1; d.max_width = 100; d.unit = 1.f / (1 << 24);
  d.g_conc = gamma_up(14, 1.0 / (1 << 24)); d.g_one = gamma_up(1, 1.0 / (1 << 24));
  d.wperm_off = (off + 3) & ~3;
  int wp = 0;
  for (int l = 0; l < 3; ++l) wp += ((dims[l] + 15) / 16) * ((dims[l + 1] + 15) / 16) * 256;
  for (int l = 0; l < 3; ++l) wp += dims[l + 1];
  d.wperm_floats = (wp + 3) & ~3;
  std::mt19937 g(1);
  std::uniform_real_distribution<float> U(-0.3f, 0.3f);
  std::vector<float> flat(d.wperm_off + d.wperm_floats, 0.f);
  for (int i = 0; i < off; ++i) flat[i] = U(g);
  // permuted block
  int p = d.wperm_off;
  for (int l = 0; l < 3; ++l) {
    const int ni = dims[l], no = dims[l + 1], tin = (ni + 15) / 16, tout = (no + 15) / 16;
    for (int jt = 0; jt < tout; ++jt)
      for (int t = 0; t < tin; ++t)
        for (int ln = 0; ln < 64; ++ln)
          for (int i = 0; i < 4; ++i) {
            const int k = 16 * t + 4 * (ln >> 4) + i, j = 16 * jt + (ln & 15);
            flat[p++] = (k < ni && j < no) ? flat[d.w_off[l] + k * no + j] : 0.f;
          }
  }
  for (int l = 0; l < 3; ++l) for (int j = 0; j < dims[l + 1]; ++j) flat[p++] = flat[d.b_off[l] + j];
  std::vector<float> lo((size_t)R * 13), hi((size_t)R * 13);
  std::uniform_int_distribution<int> B(0, 40), W(0, 9);
  for (size_t i = 0; i < lo.size(); ++i) { lo[i] = (float)B(g); hi[i] = lo[i] + (float)W(g); }
  for (int r = 0; r < R; ++r) hi[(size_t)r * 13 + 8] = lo[(size_t)r * 13 + 8];
  float *dflat, *dlo, *dhi, *o[8];
  hipMalloc(&dflat, flat.size() * 4); hipMemcpy(dflat, flat.data(), flat.size() * 4, hipMemcpyHostToDevice);
  hipMalloc(&dlo, lo.size() * 4); hipMemcpy(dlo, lo.data(), lo.size() * 4, hipMemcpyHostToDevice);
  hipMalloc(&dhi, hi.size() * 4); hipMemcpy(dhi, hi.data(), hi.size() * 4, hipMemcpyHostToDevice);
  for (int i = 0; i < 8; ++i) hipMalloc(&o[i], (size_t)R * 13 * 4);
  BoundArgs a{};
  a.flat = dflat; a.lo = dlo; a.hi = dhi; a.R = R; a.symbolic = 1;
  a.out_lb = o[0]; a.out_ub = o[1]; a.Lc = o[2]; a.L0 = o[3]; a.Le = o[4]; a.Uc = o[5]; a.U0 = o[6]; a.Ue = o[7];
  const unsigned long long fold = 1ull << 8;
  for (int w = 0; w < 3; ++w) fa_sym_try_launch(d, a, fold, 0);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  const int it = 20;
  for (int w = 0; w < it; ++w) fa_sym_try_launch(d, a, fold, 0);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  printf("{\"R\": %d, \"ms_per_launch\": %.4f, \"mrows_per_s\": %.2f}\n", R, ms / it, R / (ms / it) / 1e3);
  return 0;
}
