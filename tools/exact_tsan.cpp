// Host sanitizer harness for the multi-threaded native paths ("thread-sanitizer for
// the host solver pool").  In a bench or CLI run, 8 host threads drive the BaB runtime without
// the GIL and each confirms its candidate pairs with fa_exact::ExactChecker
// (csrc/exact_host.h); rank 0's CSV formatting core (csrc/csv_format.h) runs on a background
// thread next to them.  This harness runs both from T threads that share ONE checker (read
// only) and writes results into per-thread buffers:
//
//   g++ -std=c++17 -O1 -g -fsanitize=thread -pthread -Ifairify_amd/csrc tools/exact_tsan.cpp
//   g++ -std=c++17 -O1 -g -fsanitize=address,undefined -pthread -Ifairify_amd/csrc tools/exact_tsan.cpp
//
// Checks: no data race / memory error reported by the sanitizer; every thread's verdicts equal
// the single-threaded ones; the fp64 sign with its rounding bound never contradicts a long-double
// evaluation of the same network (ambiguous points are allowed to answer "ask").
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "csv_format.h"
#include "exact_host.h"

static int ref_sign(const fa_exact::ExactChecker& c, const double* x) {
  std::vector<long double> h(x, x + c.n0), hn;
  for (int l = 0; l < c.n_layers; ++l) {
    const int nin = c.dims[l], nout = c.dims[l + 1];
    hn.assign(nout, 0.0L);
    for (int j = 0; j < nout; ++j) {
      long double z = c.w[c.b_off[l] + j];
      for (int i = 0; i < nin; ++i) z += h[i] * (long double)c.w[c.w_off[l] + (size_t)i * nout + j];
      hn[j] = (l < c.n_layers - 1 && z < 0) ? 0.0L : z;
    }
    h.swap(hn);
  }
  return h[0] > 0 ? 1 : (h[0] < 0 ? -1 : 0);
}

int main(int argc, char** argv) {
  const int T = argc > 1 ? std::atoi(argv[1]) : 8;
  const int N = argc > 2 ? std::atoi(argv[2]) : 4000;
  std::mt19937 g(7);
  std::normal_distribution<float> nd(0.f, 0.4f);
  fa_exact::ExactChecker c;
  c.n0 = 13;
  c.dims = {13, 16, 8, 1};
  c.n_layers = 3;
  int off = 0;
  for (int l = 0; l < c.n_layers; ++l) {
    c.w_off.push_back(off);
    off += c.dims[l] * c.dims[l + 1];
    c.b_off.push_back(off);
    off += c.dims[l + 1];
  }
  for (int i = 0; i < off; ++i) c.w.push_back((double)nd(g));   // fp32 values, as the runtime's copy
  c.is_pa.assign(c.n0, 0);
  c.is_ra.assign(c.n0, 0);
  c.is_pa[8] = 1;   // Adult sex
  c.is_ra[0] = 1;   // age, tau 2 (relaxed query)
  c.tau = 2.f;
  // candidate pairs inside per-pair boxes; about half satisfy the pair constraints
  std::uniform_int_distribution<int> ui(0, 9);
  std::vector<float> pairs((size_t)N * 2 * c.n0), lo((size_t)N * c.n0), hi((size_t)N * c.n0);
  for (int k = 0; k < N; ++k) {
    for (int d = 0; d < c.n0; ++d) {
      lo[(size_t)k * c.n0 + d] = 0.f;
      hi[(size_t)k * c.n0 + d] = 9.f;
      const float x = (float)ui(g);
      float xp = x;
      if (d == 8) xp = (float)(1 - (int)x % 2);
      else if (d == 0) xp = std::fmin(9.f, x + (float)(ui(g) % 3));
      else if (ui(g) == 0 && k % 2) xp = (float)ui(g);   // breaks the shared-feature constraint
      pairs[(size_t)k * 2 * c.n0 + d] = x;
      pairs[(size_t)k * 2 * c.n0 + c.n0 + d] = xp;
    }
  }
  std::vector<int> serial(N);
  for (int k = 0; k < N; ++k)
    serial[k] = c.check(pairs.data() + (size_t)k * 2 * c.n0, lo.data() + (size_t)k * c.n0, hi.data() + (size_t)k * c.n0);
  int fails = 0, ask = 0, viol = 0;
  for (int k = 0; k < N; ++k) {
    ask += serial[k] < 0;
    viol += serial[k] == 1;
    std::vector<double> x(c.n0);
    for (int d = 0; d < c.n0; ++d) x[d] = pairs[(size_t)k * 2 * c.n0 + d];
    const int s = c.sign(x.data());
    if (s != 2 && s != ref_sign(c, x.data())) {
      if (++fails < 10) std::printf("FAIL: sign mismatch at pair %d\n", k);
    }
  }
  // T threads share the checker (const) and format CSV fields into their own strings
  std::vector<std::vector<int>> res(T, std::vector<int>(N));
  std::vector<std::string> text(T);
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      for (int k = t; k < N + t; ++k) {
        const int i = k % N;   // every thread walks all pairs from a different start
        res[t][i] = c.check(pairs.data() + (size_t)i * 2 * c.n0, lo.data() + (size_t)i * c.n0,
                            hi.data() + (size_t)i * c.n0);
        fa_csv::append_repr(text[t], 0.001 * i + t);
        fa_csv::append_round4(text[t], 1.0 / (i + 1));
        std::vector<double> v(c.n0);
        for (int d = 0; d < c.n0; ++d) v[d] = pairs[(size_t)i * 2 * c.n0 + d];
        fa_csv::append_np_vector(text[t], v.data(), c.n0);
      }
    });
#ifdef FA_TSAN_SELFTEST
  // negative control: an unsynchronised shared counter, which the thread sanitizer must report
  static int shared_hits = 0;
  for (int t = 0; t < T; ++t) th.emplace_back([] { for (int i = 0; i < 1000; ++i) ++shared_hits; });
#endif
  for (auto& x : th) x.join();
  for (int t = 0; t < T; ++t)
    for (int k = 0; k < N; ++k)
      if (res[t][k] != serial[k] && ++fails < 20) std::printf("FAIL: thread %d pair %d\n", t, k);
  std::printf("exact_tsan: %d threads x %d pairs, %d violations, %d ambiguous, %s\n", T, N, viol, ask,
              fails ? "FAILED" : "ok");
  return fails ? 1 : 0;
}
