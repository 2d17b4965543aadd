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

#include <string>
#include <vector>

#include "csv_format.h"

namespace py = pybind11;

using namespace fa_csv;


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
