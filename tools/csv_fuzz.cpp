// Host sanitizer harness for the native CSV formatting core (fairify_amd/csrc/csv_format.h).
// GPU AddressSanitizer is not available on this pool, so the host-side native code is what gets
// sanitized:  g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all
//             -Ifairify_amd/csrc tools/csv_fuzz.cpp -o /tmp/csv_fuzz && /tmp/csv_fuzz 200000
// Properties checked on random doubles of every magnitude / sign / special value:
//   * repr round-trips (strtod(repr(x)) == x, bitwise incl. -0.0) and has Python's shape
//     (contains '.', 'e', "inf" or "nan"; exponent form iff |x| < 1e-4 or >= 1e16);
//   * round4 output parses and is within 5e-5 of x (for |x| < 1e11);
//   * numpy-vector printing: balanced brackets, no line longer than 75 columns, one word per
//     element, every word parses back to the element.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "csv_format.h"

using namespace fa_csv;

static int fails = 0;
#define CHECK(c, ...)                 \
  do {                                \
    if (!(c)) {                       \
      if (++fails < 20) {             \
        std::printf("FAIL: " __VA_ARGS__); \
        std::printf("\n");            \
      }                               \
    }                                 \
  } while (0)

int main(int argc, char** argv) {
  const long n = argc > 1 ? std::atol(argv[1]) : 100000;
  std::mt19937_64 g(12345);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  const double specials[] = {0.0, -0.0, 1.0, -1.0, 1e16, 1e-4, 9.999999999999999e15, 0.0001, 0.00009999,
                             123456.0, 2.5, 0.1, 1e-300, 5e-324, 1.7976931348623157e308, INFINITY, -INFINITY, NAN};
  for (long it = 0; it < n + (long)(sizeof(specials) / sizeof(double)); ++it) {
    double x;
    if (it < (long)(sizeof(specials) / sizeof(double))) {
      x = specials[it];
    } else {
      uint64_t bits = g();
      std::memcpy(&x, &bits, 8);
      if (it % 3 == 0) x = (u(g) - 0.5) * std::pow(10.0, (double)(g() % 40) - 20.0);
      if (it % 7 == 0) x = std::round(x);
    }
    std::string s;
    append_repr(s, x);
    if (std::isnan(x)) {
      CHECK(s == "nan", "nan -> %s", s.c_str());
      continue;
    }
    const double back = std::strtod(s.c_str(), nullptr);
    CHECK(std::memcmp(&back, &x, 8) == 0 || (x == 0 && back == 0 && std::signbit(x) == std::signbit(back)),
          "repr round trip %.17g -> %s", x, s.c_str());
    if (std::isfinite(x)) {
      const bool has = s.find('.') != std::string::npos || s.find('e') != std::string::npos;
      CHECK(has, "repr shape %s", s.c_str());
      const double a = std::fabs(x);
      const bool expo = s.find('e') != std::string::npos;
      if (a != 0) CHECK(expo == (a < 1e-4 || a >= 1e16), "repr notation %.17g -> %s", x, s.c_str());
      std::string r;
      append_round4(r, x);
      const double rb = std::strtod(r.c_str(), nullptr);
      if (a < 1e11) CHECK(std::fabs(rb - x) <= 5.0001e-5 + 1e-12 * a, "round4 %.17g -> %s", x, r.c_str());
    }
  }
  // numpy vector printing
  for (long it = 0; it < n / 10; ++it) {
    const int len = 1 + (int)(g() % 40);
    std::vector<double> v(len);
    const int span = (int)(g() % 5);
    const double hi[] = {2, 10, 100, 1000, 20000};
    for (auto& e : v) e = std::floor(u(g) * hi[span]) - (it % 4 == 0 ? 3 : 0);
    std::string s;
    if (!append_np_vector(s, v.data(), len)) continue;   // exponent notation: Python fallback
    std::string t = s;
    if (!t.empty() && t.front() == '"') t = t.substr(1, t.size() - 2);
    CHECK(t.front() == '[' && t.back() == ']', "brackets %s", s.c_str());
    size_t start = 0;
    int words = 0;
    while (start < t.size()) {
      size_t nl = t.find('\n', start);
      const std::string line = t.substr(start, nl == std::string::npos ? std::string::npos : nl - start);
      CHECK(line.size() <= 75, "line too long (%zu): %s", line.size(), line.c_str());
      start = nl == std::string::npos ? t.size() : nl + 1;
    }
    const char* p = t.c_str() + 1;
    for (int k = 0; k < len; ++k) {
      char* end = nullptr;
      const double w = std::strtod(p, &end);
      CHECK(end != p && w == (double)(float)v[k], "word %d of %s", k, t.c_str());
      if (end == p) break;
      ++words;
      p = end;
      if (*p == '.') ++p;
    }
    CHECK(words == len, "word count %d vs %d", words, len);
  }
  std::printf("csv_fuzz: %s (%d failures)\n", fails ? "FAILED" : "ok", fails);
  return fails ? 1 : 0;
}
