// Native exact confirmation of BaB candidate pairs (host C++, no HIP): the pair constraints of
// the fairness query plus the logit sign of the exact network at an integer point, evaluated in
// fp64 with a rigorous rounding bound.  Only a pair whose sign the bound cannot settle goes to
// the Python rational check (engine/exact.py).  Reference semantics: a counterexample is a pair
// (x, x') that agrees on the non-protected features, differs on a protected one, stays in the
// partition box, and gets different predictions (src/AC/Verify-AC.py:127-163).
//
// Pure host code shared by the BaB runtime (csrc/bab_runtime.cpp, 8 host threads, no GIL) and
// the host sanitizer harness (tools/exact_tsan.cpp, -fsanitize=thread / address,undefined):
// every method is const and touches only the checker's immutable tables and the caller's
// buffers, so one checker may serve any number of threads.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

namespace fa_exact {

struct ExactChecker {
  int n0 = 0;
  int n_layers = 0;
  std::vector<int> dims;            // [n_layers + 1]
  std::vector<int> w_off, b_off;    // offsets into w (W_l row-major [dims[l]][dims[l+1]], then b_l)
  std::vector<double> w;            // fp64 copy of the fp32 parameters
  std::vector<char> is_pa, is_ra;   // per input dim
  float tau = 0.f;

  // sign of the exact logit at integer point x: +1 / -1, 0 when the logit's magnitude bound m
  // is exactly 0, or 2 when |z| <= the rounding bound otherwise ("ask the exact rational
  // check").  A hidden neuron whose pre-activation is certainly negative (z + err < 0) outputs
  // exactly 0 and passes on no magnitude or error; m == 0 then means every product and bias
  // feeding the logit is exactly 0 (fp64 products of fp32 weights and integers are exact and
  // non-zero unless a factor is 0; sums of non-negative terms round to 0 only when all terms
  // are 0), so the exact logit is 0 -- zero-bias networks whose ReLUs all die on a box hit this
  // constantly (random-init AC-12: 31 ms of Python rational checks per 2 000-partition item).
  int sign(const double* x) const {
    std::vector<double> h(x, x + n0), m(n0), e(n0, 0.0), hn, mn, en;
    for (int i = 0; i < n0; ++i) m[i] = std::fabs(h[i]);
    const double u = std::ldexp(1.0, -53);
    for (int l = 0; l < n_layers; ++l) {
      const int nin = dims[l], nout = dims[l + 1];
      const double* W = w.data() + w_off[l];
      const double* b = w.data() + b_off[l];
      const double ku = (nin + 3) * u;
      const double g = ku / (1.0 - ku);
      hn.assign(nout, 0.0);
      mn.assign(nout, 0.0);
      en.assign(nout, 0.0);
      for (int j = 0; j < nout; ++j) {
        double z = b[j], mm = std::fabs(b[j]), ee = g * std::fabs(b[j]);
        for (int i = 0; i < nin; ++i) {
          const double wv = W[(size_t)i * nout + j];
          z += h[i] * wv;
          mm += m[i] * std::fabs(wv);
          ee += (e[i] + g * m[i]) * std::fabs(wv);
        }
        if (l < n_layers - 1) {
          if (z + ee < 0.0) {   // certainly negative: the exact ReLU output is exactly 0
            z = 0.0;
            mm = 0.0;
            ee = 0.0;
          } else {
            z = std::max(z, 0.0);
          }
        }
        hn[j] = z;
        mn[j] = mm;
        en[j] = ee;
      }
      h.swap(hn);
      m.swap(mn);
      e.swap(en);
    }
    if (m[0] == 0.0) return 0;
    const double err = e[0] * 1.0001 + 1e-300;
    if (std::fabs(h[0]) <= err) return 2;
    return h[0] > 0 ? 1 : -1;
  }

  // pair = [x (n0 floats) | x' (n0 floats)] inside box [lo, hi]:
  // 1 violation, 0 not a violation, -1 undecided here (exact rational check)
  int check(const float* pair, const float* lo, const float* hi) const {
    std::vector<double> x(n0), xp(n0);
    for (int d = 0; d < n0; ++d) {
      x[d] = std::nearbyint((double)pair[d]);
      xp[d] = std::nearbyint((double)pair[n0 + d]);
      if (x[d] < lo[d] || x[d] > hi[d]) return 0;
      if (is_pa[d]) {
        if (x[d] == xp[d] || xp[d] < lo[d] || xp[d] > hi[d]) return 0;
      } else if (is_ra[d]) {
        if (std::fabs(x[d] - xp[d]) > tau) return 0;
      } else if (x[d] != xp[d]) {
        return 0;
      }
    }
    const int sx = sign(x.data());
    if (sx == 0) return 0;               // exact zero logit: no strict sign flip
    if (sx == 2) return -1;
    const int sp = sign(xp.data());
    if (sp == 0) return 0;
    if (sp == 2) return -1;
    return sx * sp < 0 ? 1 : 0;
  }
};

}  // namespace fa_exact
