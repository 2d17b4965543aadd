// Native formatter of the reference's 24-column per-partition CSV (src/AC/Verify-AC.py:277-315).
//
// Rank 0 of a stress run writes millions of rows (3.29 M partitions per model for stress/AC);
// the per-row Python path costs ~25 us/row and becomes the scaling bottleneck of an 8-GPU job.
// This formats the packed float64 result rows (engine/runner.py:pack) straight into CSV bytes,
// byte-identical to csv.writer(dialect='excel') over the Python values the reference writes:
//   * Python float repr (shortest round-trip digits; fixed notation for 1e-4 <= |x| < 1e16,
//     else d.ddde+XX) via std::to_chars;
//   * round(x, 4) = correctly rounded decimal (std::to_chars fixed/4 rounds the exact binary
//     value, like printf and CPython) and then repr;
//   * counterexamples as str(np.float32 array): the fixed-notation layout numpy uses for
//     integer-valued vectors ("[40.  0.  3.]", 75-column wrapping, one-space hanging indent);
//     vectors numpy would print in exponent notation are delegated to a Python callback.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

void append_repr(std::string& out, double x) {
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

void append_round4(std::string& out, double x) {
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

void append_int(std::string& out, long long v) {
  char buf[32];
  auto r = std::to_chars(buf, buf + sizeof(buf), v);
  out.append(buf, r.ptr);
}

// numpy fixed-notation print of an integer-valued float32 vector; false if numpy would use
// exponent notation or the values are not all finite integers.
bool append_np_vector(std::string& out, const double* v, int n) {
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

}  // namespace

// rows: packed [R, W] float64; layout: column indices
//   [pos, verdict, h_attempt, h_success, b_comp, s_comp, st_comp, h_comp, t_comp, sv_time, s_time,
//    hv_time, h_time, total_time, c_check, v_accurate, pruned_acc, has_cex, c1_start, c2_start]
// counts: running (sat, unsat, unknown) before the first row.  fallback(str_of_row_vector) is
// called with a float32 numpy vector for counterexamples numpy prints in exponent notation.
py::bytes format_partition_csv(py::array_t<double, py::array::c_style | py::array::forcecast> rows,
                               std::vector<int> layout, int n0, std::vector<long long> counts, py::object orig_acc,
                               py::object fallback) {
  if (rows.ndim() != 2 || layout.size() != 20 || counts.size() != 3) throw std::invalid_argument("bad arguments");
  const long long R = rows.shape(0), W = rows.shape(1);
  for (int c : layout)
    if (c < 0 || c >= W) throw std::invalid_argument("layout column out of range");
  if (layout[18] + n0 > W || layout[19] + n0 > W) throw std::invalid_argument("counterexample columns out of range");
  std::string acc;
  if (!orig_acc.is_none()) append_round4(acc, orig_acc.cast<double>());
  long long sat = counts[0], uns = counts[1], unk = counts[2];
  std::string out;
  out.reserve((size_t)R * 160);
  const double* D = rows.data();
  // formatting runs without the GIL (rank 0 formats one round while the next round's chunks
  // drive the GPU from other threads); only the exponent-notation fallback re-takes it
  {
  py::gil_scoped_release nogil;
  for (long long i = 0; i < R; ++i) {
    const double* r = D + i * W;
    const int v = (int)r[layout[1]];
    if (v == 1) ++sat; else if (v == 2) ++uns; else ++unk;
    append_int(out, (long long)r[layout[0]] + 1);
    out += v == 1 ? ",sat," : (v == 2 ? ",unsat," : ",unknown,");
    append_int(out, sat); out += ',';
    append_int(out, uns); out += ',';
    append_int(out, unk); out += ',';
    append_int(out, (long long)r[layout[2]]); out += ',';
    append_int(out, (long long)r[layout[3]]); out += ',';
    for (int k = 4; k <= 8; ++k) { append_round4(out, r[layout[k]]); out += ','; }
    for (int k = 9; k <= 13; ++k) { append_repr(out, r[layout[k]]); out += ','; }
    append_int(out, (long long)r[layout[14]]); out += ',';
    append_int(out, (long long)r[layout[15]]); out += ',';
    out += acc; out += ',';
    append_round4(out, r[layout[16]]); out += ",-,";
    if (r[layout[17]] > 0) {
      for (int which = 0; which < 2; ++which) {
        const double* vec = r + layout[18 + which];
        if (!append_np_vector(out, vec, n0)) {
          std::string t;
          {
            py::gil_scoped_acquire gil;
            py::array_t<float> a(n0);
            for (int d = 0; d < n0; ++d) a.mutable_data()[d] = (float)vec[d];
            t = fallback(a).cast<std::string>();
          }
          if (t.find('\n') != std::string::npos || t.find(',') != std::string::npos) {
            out += '"';
            out += t;
            out += '"';
          } else {
            out += t;
          }
        }
        if (which == 0) out += ',';
      }
    } else {
      out += ',';
    }
    out += "\r\n";
  }
  }
  return py::bytes(out);
}

void register_csv(py::module& m) {
  m.def("format_partition_csv", &format_partition_csv, py::arg("rows"), py::arg("layout"), py::arg("n0"),
        py::arg("counts"), py::arg("orig_acc"), py::arg("fallback"),
        "Packed result rows -> reference-format CSV bytes (engine/runner.py, report/csv_report.py)");
}
