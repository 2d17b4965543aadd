// Pure-C++ formatting core of the native CSV writer (csv_writer.cpp): Python float repr,
// round(x, 4) + repr, integers, and numpy's fixed-notation print of integer-valued float32
// vectors.  No Python dependency, so the host sanitizer harness (tools/csv_fuzz.cpp, built with
// -fsanitize=address,undefined) exercises exactly this code.
#pragma once
#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>

namespace fa_csv {

inline void append_repr(std::string& out, double x) {
  if (std::isnan(x)) { out += "nan"; return; }
  if (std::isinf(x)) { out += x > 0 ? "inf" : "-inf"; return; }
  if (std::signbit(x)) out += '-';
  if (x == 0.0) { out += "0.0"; return; }
  char buf[48];
  auto r = std::to_chars(buf, buf + sizeof(buf), std::fabs(x), std::chars_format::scientific);
  // buf = d[.ddd]e(+|-)XX : collect the significant digits and the exponent
  char digits[32];
  int nd = 0;
  const char* q = buf;
  for (; q < r.ptr && *q != 'e'; ++q)
    if (*q != '.') digits[nd++] = *q;
  int exp10 = 0;
  std::from_chars(q + 1 + (q[1] == '+' ? 1 : 0), r.ptr, exp10);
  char tmp[64];
  int k = 0;
  if (exp10 >= -4 && exp10 < 16) {
    if (exp10 >= 0) {
      if (nd <= exp10 + 1) {
        for (int i = 0; i < nd; ++i) tmp[k++] = digits[i];
        for (int i = nd; i < exp10 + 1; ++i) tmp[k++] = '0';
        tmp[k++] = '.';
        tmp[k++] = '0';
      } else {
        for (int i = 0; i <= exp10; ++i) tmp[k++] = digits[i];
        tmp[k++] = '.';
        for (int i = exp10 + 1; i < nd; ++i) tmp[k++] = digits[i];
      }
    } else {
      tmp[k++] = '0';
      tmp[k++] = '.';
      for (int i = 0; i < -exp10 - 1; ++i) tmp[k++] = '0';
      for (int i = 0; i < nd; ++i) tmp[k++] = digits[i];
    }
  } else {
    tmp[k++] = digits[0];
    if (nd > 1) {
      tmp[k++] = '.';
      for (int i = 1; i < nd; ++i) tmp[k++] = digits[i];
    }
    tmp[k++] = 'e';
    tmp[k++] = exp10 < 0 ? '-' : '+';
    const int ae = std::abs(exp10);
    if (ae < 10) tmp[k++] = '0';
    auto e = std::to_chars(tmp + k, tmp + sizeof(tmp), ae);
    k = (int)(e.ptr - tmp);
  }
  out.append(tmp, k);
}

inline void append_round4(std::string& out, double x) {
  if (!std::isfinite(x)) { append_repr(out, x); return; }
  // correctly rounded to 4 decimals (to_chars with a precision rounds the exact binary value,
  // like printf and CPython's round), then parsed back and printed as repr
  char buf[400];
  auto r = std::to_chars(buf, buf + sizeof(buf), x, std::chars_format::fixed, 4);
  double v = 0.0;
  std::from_chars(buf, r.ptr, v);
  if (v == 0.0) v = std::copysign(0.0, x);   // CPython's round keeps the sign of zero
  append_repr(out, v);
}

inline void append_int(std::string& out, long long v) {
  char buf[32];
  auto r = std::to_chars(buf, buf + sizeof(buf), v);
  out.append(buf, r.ptr);
}

// numpy fixed-notation print of an integer-valued float32 vector; false if numpy would use
// exponent notation or the values are not all finite integers.
inline bool append_np_vector(std::string& out, const double* v, int n) {
  if (n > 256) return false;
  float f[256];
  float mx = 0.f, mn = INFINITY;
  bool any = false;
  for (int i = 0; i < n; ++i) {
    f[i] = (float)v[i];
    if (!std::isfinite(f[i]) || f[i] != std::nearbyint(f[i])) return false;
    const float a = std::fabs(f[i]);
    if (a != 0.f) {
      any = true;
      mx = std::fmax(mx, a);
      mn = std::fmin(mn, a);
    }
  }
  if (any && ((double)mx >= 1e8 || (double)mn < 1e-4 || (double)(mx / mn) > 1000.0)) return false;
  char words[256][24];
  int wl[256];
  int w = 0;
  for (int i = 0; i < n; ++i) {
    auto r = std::to_chars(words[i], words[i] + 22, (long long)f[i]);
    *r.ptr = '.';
    wl[i] = (int)(r.ptr - words[i]) + 1;
    w = std::max(w, wl[i]);
  }
  // lay out: "[" + words joined by ' ', wrapped before a word that would pass column 74
  std::string txt = "[";
  int llen = 1;
  bool wrapped = false;
  for (int i = 0; i < n; ++i) {
    if (llen + w > 74 && llen > 1) {
      while (!txt.empty() && txt.back() == ' ') txt.pop_back();
      txt += "\n ";
      llen = 1;
      wrapped = true;
    }
    txt.append(w - wl[i], ' ');
    txt.append(words[i], wl[i]);
    llen += w;
    if (i != n - 1) {
      txt += ' ';
      llen += 1;
    }
  }
  txt += ']';
  if (wrapped) {
    out += '"';
    out += txt;
    out += '"';
  } else {
    out += txt;
  }
  return true;
}

}  // namespace fa_csv
