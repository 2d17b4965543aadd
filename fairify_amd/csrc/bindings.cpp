// pybind11 bindings of the fairify_amd HIP kernels (module fairify_amd._C).
//
// Tensors cross the boundary as raw device pointers (Python ints from Tensor.data_ptr()) plus
// the caller's HIP stream (torch.cuda.current_stream().cuda_stream), so the extension has no
// dependency on the torch C++ headers and launches onto whatever stream torch is using.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cmath>
#include <cstring>
#include <cstdint>
#include <stdexcept>
#include <vector>

#include "args.h"
#include "devmem.h"

namespace py = pybind11;

extern "C" int fa_bounds_launch(const NetDesc& net, BoundArgs args, hipStream_t stream);
extern "C" int fa_crown_phase_launch(const NetDesc& net, CrownPhaseArgs a, hipStream_t stream);
extern "C" size_t fa_crown_phase_bytes(const NetDesc& net);
extern "C" int fa_point_try_launch(const NetDesc& net, BoundArgs a, hipStream_t stream);
extern "C" int fa_forward_launch(const NetDesc& net, FwdArgs a, hipStream_t stream);
extern "C" int fa_sim_launch(const NetDesc& net, SimArgs a, hipStream_t stream);
extern "C" int fa_ascent_launch(const NetDesc& net, AscentArgs a, hipStream_t stream);
extern "C" int fa_certify_launch(CertArgs a, hipStream_t stream);
extern "C" int fa_falsify_launch(const NetDesc& net, FalsifyArgs a, hipStream_t stream);
extern "C" int fa_prune_masks_launch(const NetDesc& net, int P, const int* counts, const float* ub, int ub_stride,
                                     const uint8_t* sym_dead, uint8_t* code, int* cnt, hipStream_t stream);
extern "C" int fa_heuristic_launch(const NetDesc& net, int Pu, const int64_t* rows, const float* lb, const float* ub,
                                   int stride, const uint8_t* code, double q50, double qlo, double qhi, uint8_t* hnew,
                                   uint8_t* hmerged, int* hcnt, hipStream_t stream);
extern "C" int fa_agree_launch(const NetDesc& net, const float* flat, int Pm, const int64_t* rows, const float* lo,
                               const float* hi, const int64_t* pids, const uint8_t* dead, int S, uint32_t seed,
                               int* agree, hipStream_t stream);

extern "C" int fa_decode_launch(const DecodeDesc& d, const int64_t* ids, int P, const float* chunk_lo,
                                const float* chunk_hi, float* lo, float* hi, hipStream_t stream);
extern "C" int fa_trace_marker_launch(int tag, int* sink, hipStream_t stream);
extern "C" int fa_beta_launch(const NetDesc& nd, BetaArgs a, hipStream_t stream);
extern "C" int fa_beta_config(const NetDesc& nd, int* wpb, int* wtl, size_t* bytes);
extern "C" int fa_knn_launch(const float* X, int n, int d, int k, int* idx, float* dist, hipStream_t stream);
extern "C" int fa_actdiff_launch(const NetDesc& net, const float* flat, const float* x, const float* xp, int npairs,
                                 float* sum_out, hipStream_t stream);
extern "C" int fa_pack_masks_launch(const uint8_t* src, int P, int N, int stride, int sel, uint8_t* out, int NB,
                                    unsigned long long* hash, hipStream_t stream);

template <typename T>
static T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }

static float gamma_up(int k, double unit) {
  const double ku = (k + 2) * unit;
  return std::nextafter((float)(ku / (1.0 - ku)), INFINITY);
}

struct Net {
  NetDesc d;
  explicit Net(const std::vector<int>& dims, double unit) {
    if (dims.size() < 2 || dims.size() > FA_MAX_LAYERS + 1) throw std::invalid_argument("bad layer count");
    std::memset(&d, 0, sizeof(d));
    d.n_layers = (int)dims.size() - 1;
    int off = 0, noff = 0, mw = 0, mws = 0;
    for (size_t i = 0; i < dims.size(); ++i) {
      d.dims[i] = dims[i];
      mw = std::max(mw, dims[i]);
    }
    for (int l = 0; l < d.n_layers; ++l) {
      d.w_off[l] = off;
      off += dims[l] * dims[l + 1];
      d.b_off[l] = off;
      off += dims[l + 1];
      d.neuron_off[l] = noff;
      noff += dims[l + 1];
      mws = std::max(mws, dims[l] * dims[l + 1]);
      d.g_gemm[l] = gamma_up(2 * dims[l] + 1, unit);
      d.g_fwd[l] = gamma_up(dims[l] + 1, unit);
    }
    d.n_neurons = noff;
    d.n_hidden = noff - dims.back();
    d.max_width = mw;
    d.max_wsize = mws;
    d.unit = (float)unit;
    d.g_conc = gamma_up(dims[0] + 1, unit);
    d.g_one = gamma_up(1, unit);
    n_params = off;
    d.wperm_off = (off + 3) & ~3;
    int wp = 0;
    for (int l = 0; l < d.n_layers; ++l) wp += ((dims[l] + 15) / 16) * ((dims[l + 1] + 15) / 16) * 256;
    for (int l = 0; l < d.n_layers; ++l) wp += dims[l + 1];
    d.wperm_floats = (wp + 3) & ~3;
    total_floats = d.wperm_off + d.wperm_floats;
    // packed narrow-network block (ops/backend.py: pack_groups / mfma_packed_block)
    d.pack_g = 1;
    if (d.n_layers >= 2 && dims[0] <= 16 && mw <= 16) {
      int mh = 0;
      for (int l = 1; l < d.n_layers; ++l) mh = std::max(mh, dims[l]);
      d.pack_g = mh <= 4 ? 4 : (mh <= 8 ? 2 : 1);   // box stride 16 / pack_g: a multiple of 4
    }
    d.pack_off = total_floats;
    d.pack_floats = 0;
    if (d.pack_g > 1) {
      d.pack_floats = d.pack_g * 256 + (d.n_layers - 1) * 256 + d.n_layers * 16;
      total_floats += d.pack_floats;
    }
    // backward operand order block (ops/backend.py: mfma_back_block)
    d.wback_off = total_floats;
    int wb = 0;
    for (int l = 0; l < d.n_layers; ++l) wb += ((dims[l] + 15) / 16) * ((dims[l + 1] + 15) / 16) * 256;
    d.wback_floats = wb;
    total_floats += wb;
  }
  int n_params;
  int total_floats;
};

const NetDesc& fa_net_desc(py::handle h) { return h.cast<const Net&>().d; }
void register_bab(py::module& m);
void register_relu(py::module& m);
void register_beta(py::module& m);
extern "C" int fa_crown_launch(const NetDesc& net, BoundArgs a, hipStream_t stream);
extern "C" int fa_refine_launch(const NetDesc& net, BoundArgs a, hipStream_t stream);
extern "C" int fa_backward_launch(const NetDesc& net, BoundArgs a, hipStream_t stream);
extern "C" int fa_refine_crown_launch(const NetDesc& net, BoundArgs a, hipStream_t stream);
void register_csv(py::module& m);

static void check(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string(what) + " launch failed, code " + std::to_string(rc));
}

PYBIND11_MODULE(_C, m) {
  m.doc() = "fairify_amd CDNA4 (gfx950) kernels";
  py::class_<Net>(m, "Net")
      .def(py::init<const std::vector<int>&, double>())
      .def_readonly("n_params", &Net::n_params)
      .def_readonly("total_floats", &Net::total_floats)
      .def_property_readonly("wperm_off", [](const Net& n) { return n.d.wperm_off; })
      .def_property_readonly("pack_g", [](const Net& n) { return n.d.pack_g; })
      .def_property_readonly("pack_off", [](const Net& n) { return n.d.pack_off; })
      .def_property_readonly("n_hidden", [](const Net& n) { return n.d.n_hidden; })
      .def_property_readonly("n_neurons", [](const Net& n) { return n.d.n_neurons; });

  m.def("bounds", [](const Net& net, uintptr_t flat, uintptr_t lo, uintptr_t hi, uintptr_t dead_in, int R,
                     int symbolic, uintptr_t out_lb, uintptr_t out_ub, uintptr_t Lc, uintptr_t L0, uintptr_t Le,
                     uintptr_t Uc, uintptr_t U0, uintptr_t Ue, uintptr_t layer_lb, uintptr_t layer_ub,
                     uintptr_t dead_out, int G, uintptr_t stream, unsigned long long fold, uintptr_t phase_in,
                     uintptr_t infeas) {
    NetDesc d = net.d;
    BoundArgs a{};
    a.flat = P<const float>(flat);
    a.lo = P<const float>(lo);
    a.hi = P<const float>(hi);
    a.dead_in = P<const uint8_t>(dead_in);
    a.R = R;
    a.symbolic = symbolic;
    a.G = G;
    a.out_lb = P<float>(out_lb);
    a.out_ub = P<float>(out_ub);
    a.Lc = P<float>(Lc); a.L0 = P<float>(L0); a.Le = P<float>(Le);
    a.Uc = P<float>(Uc); a.U0 = P<float>(U0); a.Ue = P<float>(Ue);
    a.layer_lb = P<float>(layer_lb);
    a.layer_ub = P<float>(layer_ub);
    a.dead_out = P<uint8_t>(dead_out);
    a.fold = fold;
    a.phase_in = P<const int8_t>(phase_in);
    a.infeas = P<uint8_t>(infeas);
    check(fa_bounds_launch(d, a, (hipStream_t)stream), "bounds");
  }, py::arg("net"), py::arg("flat"), py::arg("lo"), py::arg("hi"), py::arg("dead_in"), py::arg("R"),
     py::arg("symbolic"), py::arg("out_lb"), py::arg("out_ub"), py::arg("Lc"), py::arg("L0"), py::arg("Le"),
     py::arg("Uc"), py::arg("U0"), py::arg("Ue"), py::arg("layer_lb"), py::arg("layer_ub"), py::arg("dead_out"),
     py::arg("G"), py::arg("stream"), py::arg("fold") = 0ull, py::arg("phase_in") = 0, py::arg("infeas") = 0);

  // ReLU-phase backward bounds (relu.hip), refining a preceding phase-aware `bounds` call in place
  m.def("crown_phase", [](const Net& net, uintptr_t flat, uintptr_t lo, uintptr_t hi, int R, uintptr_t phase,
                          uintptr_t layer_lb, uintptr_t layer_ub, uintptr_t infeas, uintptr_t out_lb, uintptr_t out_ub,
                          uintptr_t Lc, uintptr_t L0, uintptr_t Le, uintptr_t Uc, uintptr_t U0, uintptr_t Ue,
                          uintptr_t split, uintptr_t score, uintptr_t low, uintptr_t stream) {
    CrownPhaseArgs a{};
    a.flat = P<const float>(flat);
    a.lo = P<const float>(lo);
    a.hi = P<const float>(hi);
    a.R = R;
    a.phase = P<const int8_t>(phase);
    a.layer_lb = P<const float>(layer_lb);
    a.layer_ub = P<const float>(layer_ub);
    a.infeas = P<const uint8_t>(infeas);
    a.out_lb = P<float>(out_lb);
    a.out_ub = P<float>(out_ub);
    a.Lc = P<float>(Lc); a.L0 = P<float>(L0); a.Le = P<float>(Le);
    a.Uc = P<float>(Uc); a.U0 = P<float>(U0); a.Ue = P<float>(Ue);
    a.split = P<int>(split);
    a.score = P<float>(score);
    a.low = P<float>(low);
    const int rc = fa_crown_phase_launch(net.d, a, (hipStream_t)stream);
    if (rc != 0) throw std::runtime_error("crown_phase launch failed, code " + std::to_string(rc));
  });

  // does the ReLU-phase backward kernel hold this network (layers <= 256 wide, LDS <= 160 KB)?
  m.def("relu_fits", [](const Net& net) { return fa_crown_phase_bytes(net.d) > 0; });

  // backward output bounds refining forms/out bounds written by a preceding `bounds` call
  m.def("crown", [](const Net& net, uintptr_t flat, uintptr_t lo, uintptr_t hi, uintptr_t dead_in, int R,
                    uintptr_t out_lb, uintptr_t out_ub, uintptr_t Lc, uintptr_t L0, uintptr_t Le, uintptr_t Uc,
                    uintptr_t U0, uintptr_t Ue, uintptr_t layer_lb, uintptr_t layer_ub, uintptr_t stream) {
    BoundArgs a{};
    a.flat = P<const float>(flat);
    a.lo = P<const float>(lo);
    a.hi = P<const float>(hi);
    a.dead_in = P<const uint8_t>(dead_in);
    a.R = R;
    a.out_lb = P<float>(out_lb);
    a.out_ub = P<float>(out_ub);
    a.Lc = P<float>(Lc); a.L0 = P<float>(L0); a.Le = P<float>(Le);
    a.Uc = P<float>(Uc); a.U0 = P<float>(U0); a.Ue = P<float>(Ue);
    a.layer_lb = P<float>(layer_lb);
    a.layer_ub = P<float>(layer_ub);
    check(fa_crown_launch(net.d, a, (hipStream_t)stream), "crown");
  });

  // back-substituted hidden-layer bounds (refine.hip), tightening layer_lb / layer_ub of a preceding
  // symbolic `bounds` call in place; returns the launch code (0 done, -1 shape not supported)
  m.def("refine", [](const Net& net, uintptr_t flat, uintptr_t lo, uintptr_t hi, uintptr_t dead_in, int R,
                     uintptr_t layer_lb, uintptr_t layer_ub, uintptr_t stream, uintptr_t phase, uintptr_t infeas) {
    BoundArgs a{};
    a.flat = P<const float>(flat);
    a.lo = P<const float>(lo);
    a.hi = P<const float>(hi);
    a.dead_in = P<const uint8_t>(dead_in);
    a.R = R;
    a.layer_lb = P<float>(layer_lb);
    a.layer_ub = P<float>(layer_ub);
    a.phase_in = P<const int8_t>(phase);   // ReLU-phase rows [R, n_hidden] (+1 / -1 fixed, 0 free)
    a.infeas = P<uint8_t>(infeas);         // [R] set to 1 where a refined bound contradicts a phase
    const int rc = fa_refine_launch(net.d, a, (hipStream_t)stream);
    if (rc < -1) throw std::runtime_error("refine launch failed, code " + std::to_string(rc));
    return rc;
  }, py::arg("net"), py::arg("flat"), py::arg("lo"), py::arg("hi"), py::arg("dead_in"), py::arg("R"),
     py::arg("layer_lb"), py::arg("layer_ub"), py::arg("stream"), py::arg("phase") = 0, py::arg("infeas") = 0);

  // refined hidden-layer bounds + the logit's backward pass in one launch (what the BaB runtime runs
  // for BaBConfig.refine level 1), tightening a preceding symbolic `bounds` call in place
  m.def("refine_crown", [](const Net& net, uintptr_t flat, uintptr_t lo, uintptr_t hi, uintptr_t dead_in, int R,
                           uintptr_t out_lb, uintptr_t out_ub, uintptr_t Lc, uintptr_t L0, uintptr_t Le, uintptr_t Uc,
                           uintptr_t U0, uintptr_t Ue, uintptr_t layer_lb, uintptr_t layer_ub, uintptr_t stream) {
    BoundArgs a{};
    a.flat = P<const float>(flat);
    a.lo = P<const float>(lo);
    a.hi = P<const float>(hi);
    a.dead_in = P<const uint8_t>(dead_in);
    a.R = R;
    a.out_lb = P<float>(out_lb); a.out_ub = P<float>(out_ub);
    a.Lc = P<float>(Lc); a.L0 = P<float>(L0); a.Le = P<float>(Le);
    a.Uc = P<float>(Uc); a.U0 = P<float>(U0); a.Ue = P<float>(Ue);
    a.layer_lb = P<float>(layer_lb);
    a.layer_ub = P<float>(layer_ub);
    const int rc = fa_refine_crown_launch(net.d, a, (hipStream_t)stream);
    if (rc < -1) throw std::runtime_error("refine_crown launch failed, code " + std::to_string(rc));
    return rc;
  });

  // every neuron's bounds and the logit's forms by back-substitution alone (refine.hip, mode FULL);
  // layer_lb / layer_ub may be 0.  Returns the launch code (0 done, -1 shape not supported)
  m.def("backward_bounds", [](const Net& net, uintptr_t flat, uintptr_t lo, uintptr_t hi, uintptr_t dead_in, int R,
                              uintptr_t out_lb, uintptr_t out_ub, uintptr_t Lc, uintptr_t L0, uintptr_t Le,
                              uintptr_t Uc, uintptr_t U0, uintptr_t Ue, uintptr_t layer_lb, uintptr_t layer_ub,
                              uintptr_t stream) {
    BoundArgs a{};
    a.flat = P<const float>(flat);
    a.lo = P<const float>(lo);
    a.hi = P<const float>(hi);
    a.dead_in = P<const uint8_t>(dead_in);
    a.R = R;
    a.out_lb = P<float>(out_lb); a.out_ub = P<float>(out_ub);
    a.Lc = P<float>(Lc); a.L0 = P<float>(L0); a.Le = P<float>(Le);
    a.Uc = P<float>(Uc); a.U0 = P<float>(U0); a.Ue = P<float>(Ue);
    a.layer_lb = P<float>(layer_lb);
    a.layer_ub = P<float>(layer_ub);
    const int rc = fa_backward_launch(net.d, a, (hipStream_t)stream);
    if (rc < -1) throw std::runtime_error("backward_bounds launch failed, code " + std::to_string(rc));
    return rc;
  });

  m.def("point_bounds", [](const Net& net, uintptr_t flat, uintptr_t x, uintptr_t dead_in, int R, uintptr_t out_lb,
                           uintptr_t out_ub, uintptr_t stream) {
    BoundArgs a{};
    a.flat = P<const float>(flat);
    a.lo = P<const float>(x);
    a.hi = P<const float>(x);
    a.dead_in = P<const uint8_t>(dead_in);
    a.R = R;
    a.out_lb = P<float>(out_lb);
    a.out_ub = P<float>(out_ub);
    int rc = fa_point_try_launch(net.d, a, (hipStream_t)stream);
    if (rc < 0) check(-rc, "point_bounds");
    if (rc == 0) check(fa_bounds_launch(net.d, a, (hipStream_t)stream), "point_bounds(ibp)");
  });

  m.def("forward", [](const Net& net, uintptr_t flat, uintptr_t x, int B, uintptr_t dead, uintptr_t out,
                      uintptr_t stream) {
    FwdArgs a{};
    a.flat = P<const float>(flat);
    a.x = P<const float>(x);
    a.B = B;
    a.dead = P<const uint8_t>(dead);
    a.out = P<float>(out);
    check(fa_forward_launch(net.d, a, (hipStream_t)stream), "forward");
  });

  m.def("sim", [](const Net& net, uintptr_t flat, uintptr_t lo, uintptr_t hi, uintptr_t pids, int Pn, int n_samples,
                  uint32_t seed, int V, const std::vector<int>& pa, uintptr_t values, int Pp, uintptr_t pairs,
                  const std::vector<int>& ra, int tau, uintptr_t counts, uintptr_t found, uintptr_t wit_x,
                  uintptr_t wit_xp, uintptr_t z0, uintptr_t keys, int split, uintptr_t stream) {
    if (pa.size() > FA_MAX_PA || ra.size() > FA_MAX_RA) throw std::invalid_argument("too many PA/RA dims");
    if (split < 1 || (split > 1 && !keys)) throw std::invalid_argument("sim: split > 1 needs a keys buffer");
    SimArgs a{};
    a.flat = P<const float>(flat);
    a.lo = P<const float>(lo);
    a.hi = P<const float>(hi);
    a.pids = P<const int64_t>(pids);
    a.P = Pn;
    a.n_samples = n_samples;
    a.seed = seed;
    a.V = V;
    a.npa = (int)pa.size();
    for (size_t i = 0; i < pa.size(); ++i) a.pa_idx[i] = pa[i];
    a.values = P<const int64_t>(values);
    a.Pp = Pp;
    a.pairs = P<const int64_t>(pairs);
    a.nra = (int)ra.size();
    for (size_t i = 0; i < ra.size(); ++i) a.ra_idx[i] = ra[i];
    a.tau = tau;
    a.counts = P<int>(counts);
    a.found = P<uint8_t>(found);
    a.wit_x = P<float>(wit_x);
    a.wit_xp = P<float>(wit_xp);
    a.z0 = P<float>(z0);
    a.keys = P<int>(keys);
    a.split = split;
    check(fa_sim_launch(net.d, a, (hipStream_t)stream), "sim");
  });

  // returns false if the partition's candidate rows do not fit in LDS (caller keeps PyTorch)
  m.def("ascent", [](const Net& net, uintptr_t flat, uintptr_t lo, uintptr_t hi, uintptr_t x0, uintptr_t f0,
                     uintptr_t q0, int Pn, int K, int iters, int V, const std::vector<int>& pa, uintptr_t values,
                     int Pp, uintptr_t pairs, const std::vector<int>& free_dims, uintptr_t found, uintptr_t wit_x,
                     uintptr_t wit_xp, uintptr_t stream) {
    if (pa.size() > FA_MAX_PA || free_dims.size() > 64) throw std::invalid_argument("too many PA/free dims");
    AscentArgs a{};
    a.flat = P<const float>(flat);
    a.lo = P<const float>(lo);
    a.hi = P<const float>(hi);
    a.x0 = P<const float>(x0);
    a.f0 = P<const float>(f0);
    a.q0 = P<const int>(q0);
    a.P = Pn; a.K = K; a.iters = iters; a.V = V;
    a.npa = (int)pa.size();
    for (size_t i = 0; i < pa.size(); ++i) a.pa_idx[i] = pa[i];
    a.values = P<const int64_t>(values);
    a.Pp = Pp;
    a.pairs = P<const int64_t>(pairs);
    a.nfree = (int)free_dims.size();
    for (size_t i = 0; i < free_dims.size(); ++i) a.free_idx[i] = free_dims[i];
    a.found = P<uint8_t>(found);
    a.wit_x = P<float>(wit_x);
    a.wit_xp = P<float>(wit_xp);
    const int rc = fa_ascent_launch(net.d, a, (hipStream_t)stream);
    if (rc == -1) return false;
    check(rc, "ascent");
    return true;
  });

  // fused residual falsifier; returns false when the network shape is not supported (caller
  // keeps the PyTorch path)
  m.def("falsify", [](const Net& net, uintptr_t flat, uintptr_t lo, uintptr_t hi, uintptr_t pids, int Pn,
                      int n_samples, int n_local, uint32_t seed, int V, const std::vector<int>& pa, uintptr_t values,
                      int Pp, uintptr_t pairs, int walk_k, int walk_steps, int K, int iters,
                      const std::vector<int>& free_dims, uintptr_t found, uintptr_t wit_x, uintptr_t wit_xp,
                      uintptr_t how, uintptr_t stream, const std::vector<int>& ra, int tau, uint32_t dseed) {
    if (pa.size() > FA_MAX_PA || free_dims.size() > 64 || ra.size() > FA_MAX_RA)
      throw std::invalid_argument("too many PA/RA/free dims");
    FalsifyArgs a{};
    a.flat = P<const float>(flat);
    a.lo = P<const float>(lo);
    a.hi = P<const float>(hi);
    a.pids = P<const int64_t>(pids);
    a.P = Pn; a.n_samples = n_samples; a.n_local = n_local; a.seed = seed;
    a.V = V;
    a.npa = (int)pa.size();
    for (size_t i = 0; i < pa.size(); ++i) a.pa_idx[i] = pa[i];
    a.values = P<const int64_t>(values);
    a.Pp = Pp;
    a.pairs = P<const int64_t>(pairs);
    a.walk_k = walk_k; a.walk_steps = walk_steps; a.K = K; a.iters = iters;
    a.nfree = (int)free_dims.size();
    for (size_t i = 0; i < free_dims.size(); ++i) a.free_idx[i] = free_dims[i];
    a.found = P<uint8_t>(found);
    a.wit_x = P<float>(wit_x);
    a.wit_xp = P<float>(wit_xp);
    a.how = P<int8_t>(how);
    a.nra = tau > 0 ? (int)ra.size() : 0;
    for (int i = 0; i < a.nra; ++i) a.ra_idx[i] = ra[i];
    a.tau = tau;
    a.dseed = dseed;
    const int rc = fa_falsify_launch(net.d, a, (hipStream_t)stream);
    if (rc == 0) return false;
    if (rc < 0) check(-rc, "falsify");
    return true;
  });

  m.def("prune_masks", [](const Net& net, int Pn, uintptr_t counts, uintptr_t ub, int ub_stride, uintptr_t sym_dead,
                          uintptr_t code, uintptr_t cnt, uintptr_t stream) {
    check(fa_prune_masks_launch(net.d, Pn, P<const int>(counts), P<const float>(ub), ub_stride,
                                P<const uint8_t>(sym_dead), P<uint8_t>(code), P<int>(cnt), (hipStream_t)stream),
          "prune_masks");
  });

  m.def("heuristic", [](const Net& net, int Pu, uintptr_t rows, uintptr_t lb, uintptr_t ub, int stride, uintptr_t code,
                        double q50, double qlo, double qhi, uintptr_t hnew, uintptr_t hmerged, uintptr_t hcnt,
                        uintptr_t stream) {
    check(fa_heuristic_launch(net.d, Pu, P<const int64_t>(rows), P<const float>(lb), P<const float>(ub), stride,
                              P<const uint8_t>(code), q50, qlo, qhi, P<uint8_t>(hnew), P<uint8_t>(hmerged),
                              P<int>(hcnt), (hipStream_t)stream),
          "heuristic");
  });

  // returns false when the network shape is not supported (caller keeps the PyTorch path)
  m.def("agree", [](const Net& net, uintptr_t flat, int Pm, uintptr_t rows, uintptr_t lo, uintptr_t hi, uintptr_t pids,
                    uintptr_t dead, int S, uint32_t seed, uintptr_t agree, uintptr_t stream) {
    const int rc = fa_agree_launch(net.d, P<const float>(flat), Pm, P<const int64_t>(rows), P<const float>(lo),
                                   P<const float>(hi), P<const int64_t>(pids), P<const uint8_t>(dead), S, seed,
                                   P<int>(agree), (hipStream_t)stream);
    if (rc == 0) return false;
    if (rc < 0) check(-rc, "agree");
    return true;
  });

  m.def("certify", [](int Nn, int n0, int V, int Pp, int norient, std::vector<uintptr_t> fx, std::vector<uintptr_t> fxp,
                      uintptr_t xlo, uintptr_t xhi, uintptr_t xplo, uintptr_t xphi, uintptr_t pairs, uintptr_t values,
                      const std::vector<int>& pa, const std::vector<int>& ra, double tau, uintptr_t shared,
                      double unit, double gmarg, uintptr_t gmin, uintptr_t tstar, uintptr_t open, uintptr_t score,
                      uintptr_t split_dim, uintptr_t cand_x, uintptr_t cand_xp, uintptr_t cand_v, uintptr_t cand_o,
                      uintptr_t scores, uintptr_t leaf, uintptr_t stream) {
    if (pa.size() > FA_CMAX_PA || ra.size() > FA_MAX_RA) throw std::invalid_argument("too many PA/RA dims");
    if (fx.size() != 8 || fxp.size() != 8) throw std::invalid_argument("need 8 form pointers (6 forms + lb/ub)");
    CertArgs a{};
    a.Nn = Nn; a.n0 = n0; a.V = V; a.Pp = Pp; a.norient = norient;
    a.Lc = P<const float>(fx[0]); a.L0 = P<const float>(fx[1]); a.Le = P<const float>(fx[2]);
    a.Uc = P<const float>(fx[3]); a.U0 = P<const float>(fx[4]); a.Ue = P<const float>(fx[5]);
    a.olb = P<const float>(fx[6]); a.oub = P<const float>(fx[7]);
    a.Lcp = P<const float>(fxp[0]); a.L0p = P<const float>(fxp[1]); a.Lep = P<const float>(fxp[2]);
    a.Ucp = P<const float>(fxp[3]); a.U0p = P<const float>(fxp[4]); a.Uep = P<const float>(fxp[5]);
    a.olbp = P<const float>(fxp[6]); a.oubp = P<const float>(fxp[7]);
    a.xlo = P<const float>(xlo); a.xhi = P<const float>(xhi);
    a.xplo = P<const float>(xplo); a.xphi = P<const float>(xphi);
    a.pairs = P<const int64_t>(pairs);
    a.values = P<const int64_t>(values);
    a.npa = (int)pa.size();
    for (size_t i = 0; i < pa.size(); ++i) a.pa_idx[i] = pa[i];
    a.nra = (int)ra.size();
    for (size_t i = 0; i < ra.size(); ++i) a.ra_idx[i] = ra[i];
    a.tau = (float)tau;
    a.shared = P<const uint8_t>(shared);
    a.unit = (float)unit;
    a.gmarg = std::nextafter((float)gmarg, INFINITY);
    a.gmin = P<float>(gmin); a.tstar = P<float>(tstar);
    a.open = P<uint8_t>(open); a.score = P<float>(score); a.split_dim = P<int64_t>(split_dim);
    a.cand_x = P<float>(cand_x); a.cand_xp = P<float>(cand_xp);
    a.cand_v = P<int64_t>(cand_v); a.cand_o = P<int64_t>(cand_o);
    a.scores = P<float>(scores); a.leaf = P<uint8_t>(leaf);
    check(fa_certify_launch(a, (hipStream_t)stream), "certify");
  });

  m.def("decode", [](std::vector<int> radix, std::vector<long long> div, std::vector<int> chunk_off,
                     std::vector<float> base_lo, std::vector<float> base_hi, uintptr_t ids, int Pn,
                     uintptr_t chunk_lo, uintptr_t chunk_hi, uintptr_t lo, uintptr_t hi, uintptr_t stream) {
    const size_t n0 = radix.size();
    if (n0 == 0 || n0 > FA_DECODE_MAX_DIMS || div.size() != n0 || chunk_off.size() != n0 || base_lo.size() != n0 ||
        base_hi.size() != n0)
      throw std::invalid_argument("decode: descriptor sizes");
    DecodeDesc d{};
    d.n0 = (int)n0;
    for (size_t k = 0; k < n0; ++k) {
      if (radix[k] < 0 || (radix[k] > 0 && div[k] <= 0)) throw std::invalid_argument("decode: radix/div");
      d.radix[k] = radix[k];
      d.div[k] = div[k];
      d.chunk_off[k] = chunk_off[k];
      d.base_lo[k] = base_lo[k];
      d.base_hi[k] = base_hi[k];
    }
    check(fa_decode_launch(d, P<const int64_t>(ids), Pn, P<const float>(chunk_lo), P<const float>(chunk_hi),
                           P<float>(lo), P<float>(hi), (hipStream_t)stream),
          "decode");
  });
  m.def("pack_masks", [](uintptr_t src, int Pn, int N, int stride, int sel, uintptr_t out, int NB, uintptr_t hash,
                         uintptr_t stream) {
    check(fa_pack_masks_launch(P<const uint8_t>(src), Pn, N, stride, sel, P<uint8_t>(out), NB,
                               P<unsigned long long>(hash), (hipStream_t)stream),
          "pack_masks");
  });
  m.def("knn", [](uintptr_t X, int n, int d, int k, uintptr_t idx, uintptr_t dist, uintptr_t stream) {
    check(fa_knn_launch(P<const float>(X), n, d, k, P<int>(idx), P<float>(dist), (hipStream_t)stream), "knn");
  });
  m.def("actdiff", [](const Net& net, uintptr_t flat, uintptr_t x, uintptr_t xp, int npairs, uintptr_t sum_out,
                      uintptr_t stream) {
    check(fa_actdiff_launch(net.d, P<const float>(flat), P<const float>(x), P<const float>(xp), npairs,
                            P<float>(sum_out), (hipStream_t)stream),
          "actdiff");
  });
  m.def("trace_marker", [](int tag, uintptr_t sink, uintptr_t stream) {
    check(fa_trace_marker_launch(tag, P<int>(sink), (hipStream_t)stream), "trace_marker");
  });
  m.def("beta_level", [](const Net& net, uintptr_t flat, uintptr_t wt, int R, std::vector<int> pa, uintptr_t lo,
                         uintptr_t hi, uintptr_t va, uintptr_t vb, uintptr_t LBA, uintptr_t UBA, uintptr_t LBB,
                         uintptr_t UBB, uintptr_t phA, uintptr_t phB, uintptr_t par, uintptr_t t, uintptr_t scratch,
                         int iters, float lr_a, float lr_b, float lr_t, float decay, int lookahead, int beta_pos,
                         int stall,
                         uintptr_t bound, uintptr_t split, uintptr_t xstar, uintptr_t binit,
                         unsigned long long ramask, uintptr_t plo, uintptr_t phi, uintptr_t xpstar, uintptr_t gtie,
                         float tau, uintptr_t osg, uintptr_t stream) {
    if (pa.size() > FA_MAX_PA) throw std::invalid_argument("beta_level: too many PA dims");
    for (size_t q = 0; q < pa.size(); ++q)
      if (pa[q] < 0 || pa[q] >= net.d.dims[0] || (q && pa[q] <= pa[q - 1]))
        throw std::invalid_argument("beta_level: PA dims must be increasing input indices");
    BetaArgs a;
    std::memset(&a, 0, sizeof(a));
    a.flat = P<const float>(flat);
    a.wt = P<const float>(wt);
    a.R = R;
    a.npa = (int)pa.size();
    for (size_t q = 0; q < pa.size(); ++q) a.pa_idx[q] = pa[q];
    a.lo = P<const float>(lo);
    a.hi = P<const float>(hi);
    a.va = P<const float>(va);
    a.vb = P<const float>(vb);
    a.LBA = P<const float>(LBA);
    a.UBA = P<const float>(UBA);
    a.LBB = P<const float>(LBB);
    a.UBB = P<const float>(UBB);
    a.phA = P<const int8_t>(phA);
    a.phB = P<const int8_t>(phB);
    a.par = P<float>(par);
    a.t = P<float>(t);
    a.scratch = P<float>(scratch);
    a.iters = iters;
    a.lr_a = lr_a;
    a.lr_b = lr_b;
    a.lr_t = lr_t;
    a.decay = decay;
    a.lookahead = lookahead;
    a.beta_pos = beta_pos;
    a.stall = stall & 1;        // bit 1: primal-gap branching (ops/hip.py:beta_level)
    a.pgap = (stall >> 1) & 3;
    a.feas = (stall >> 3) & 1;  // bit 3: the infeasibility pass (scratch [R, 16, NH])
    a.bound = P<double>(bound);
    a.split = P<int>(split);
    a.xstar = P<float>(xstar);
    a.binit = P<float>(binit);
    a.ramask = ramask;
    a.plo = P<const float>(plo);
    a.phi = P<const float>(phi);
    a.xpstar = P<float>(xpstar);
    a.gtie = P<float>(gtie);
    a.tau = tau;
    a.osg = P<const int8_t>(osg);
    if ((net.d.dims[0] < 64 && (ramask >> net.d.dims[0])) || (ramask && (!plo || !phi)))
      throw std::invalid_argument("beta_level: RA mask beyond the inputs or no x' box");
    return fa_beta_launch(net.d, a, reinterpret_cast<hipStream_t>(stream));
  });
  m.def("beta_config", [](const Net& net) {
    int w = 0, t = 0;
    size_t b = 0;
    const int rc = fa_beta_config(net.d, &w, &t, &b);
    return py::make_tuple(rc, w, t, b);
  });
  m.def("beta_fits", [](const Net& net) {
    int w = 0, t = 0;
    size_t b = 0;
    return fa_beta_config(net.d, &w, &t, &b) == 0;
  });
  m.def("arch", []() { return std::string("gfx950"); });
  // raise the dynamic-LDS limit of every registered kernel once (common.h); Backend construction
  // calls it before any host thread launches.  0 on success.
  m.def("prepare_lds", [] { return fa_lds_prepare(); });
  m.def("lds_registered", [] { return (int)fa_lds_registry().size(); });
  register_bab(m);
  register_relu(m);
  register_beta(m);
  // caching allocator of the native runtimes (devmem.h): hipFree / hipHostFree calls reaching the
  // driver stay 0 in steady state
  m.def("mem_stats", [] {
    const fa_mem::Stats s = fa_mem::stats();
    py::dict d;
    d["dev_cached_bytes"] = s.dev_cached_bytes;
    d["dev_live_bytes"] = s.dev_live_bytes;
    d["host_cached_bytes"] = s.host_cached_bytes;
    d["host_live_bytes"] = s.host_live_bytes;
    d["dev_mallocs"] = s.dev_mallocs;
    d["dev_hits"] = s.dev_hits;
    d["host_mallocs"] = s.host_mallocs;
    d["host_hits"] = s.host_hits;
    d["driver_frees"] = s.driver_frees;
    return d;
  });
  m.def("mem_release_cached", [] { fa_mem::release_cached(); });
  register_csv(m);
}
