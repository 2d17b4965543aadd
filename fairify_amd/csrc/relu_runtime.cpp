// Native ReLU-phase branch-and-bound driver (stage "relu", engine/relu_bab.py: the torch path is
// the reference semantics).  Host loop over BFS levels of device-resident node pools; per level
// and sub-batch of nodes:
//   rows (PA values per row) -> forward symbolic bounds with the rows' ReLU phases (symbolic.hip)
//   -> every-layer backward bounds (relu.hip: fa_crown_phase) -> node certificate + vertex pair +
//   branching decision -> rigorous point bounds of the vertex pairs -> candidates / children
// then one settle kernel and ONE host synchronisation; candidate pairs are confirmed exactly on
// the host (fp64 with a rigorous bound, exact_host.h; undecided signs -> Python rational check).
#include <hip/hip_runtime.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "args.h"
#include "devmem.h"
#include "exact_host.h"

namespace py = pybind11;

extern "C" int fa_bounds_launch(const NetDesc& net, BoundArgs args, hipStream_t stream);
extern "C" int fa_point_try_launch(const NetDesc& net, BoundArgs a, hipStream_t stream);
extern "C" int fa_crown_phase_launch(const NetDesc& net, CrownPhaseArgs a, hipStream_t stream);
extern "C" int fa_refine_launch(const NetDesc& net, BoundArgs a, hipStream_t stream);
extern "C" int fa_relu_rows_launch(ReluLevelArgs a, hipStream_t stream);
extern "C" int fa_relu_cert_launch(ReluLevelArgs a, hipStream_t stream);
extern "C" int fa_relu_split_launch(ReluLevelArgs a, hipStream_t stream);
extern "C" int fa_relu_settle_launch(int P, int8_t* status, const int* part_nodes, int* nodes_start, int* counters,
                                     int* host_counts, hipStream_t stream);
extern "C" int fa_relu_reset_launch(int* counters, hipStream_t stream);

const NetDesc& fa_net_desc(py::handle net);

namespace {

void rck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
void rckl(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string(what) + " launch failed, code " + std::to_string(rc));
}

template <typename T>
using RBuf = fa_mem::DevBuf<T>;

float rgamma(int k, double unit) {
  const double ku = (k + 2) * unit;
  return std::nextafter((float)(ku / (1.0 - ku)), INFINITY);
}

}  // namespace

class ReluRuntime {
 public:
  ReluRuntime(py::handle net, uintptr_t flat, std::vector<int> pa, std::vector<float> values_f,
              std::vector<int64_t> pairs, int capacity, int batch_nodes, double unit, int refine,
              std::vector<int> ra, double tau, int norient)
      : net_(fa_net_desc(net)), flat_((const float*)flat), pa_(std::move(pa)), cap_(capacity), batch_(batch_nodes),
        unit_(unit), refine_(refine), ra_(std::move(ra)), tau_((float)tau) {
    n0_ = net_.dims[0];
    nh_ = net_.n_hidden;
    npa_ = (int)pa_.size();
    if (npa_ == 0 || npa_ > FA_CMAX_PA) throw std::invalid_argument("bad PA");
    // relaxed queries (x' RA box per node): at most FA_MAX_RA dims, none of them a PA dim
    relaxed_ = !ra_.empty() && tau_ > 0.f;
    if (!relaxed_) ra_.clear();
    if ((int)ra_.size() > FA_MAX_RA) throw std::invalid_argument("bad RA");
    for (int d : ra_) {
      if (d < 0 || d >= n0_) throw std::invalid_argument("RA dim out of range");
      for (int k : pa_)
        if (k == d) throw std::invalid_argument("RA dim is a PA dim");
    }
    V_ = (int)(values_f.size() / npa_);
    // relaxed queries, norient = 2: both orientations are roots of the same search -- every ordered
    // pair appears twice in the table, the second copy (index >= neg_from_) ruling out the reverse
    // orientation N(x, va) > 0 > N(x', vb) (relu.hip reads the negated logit's forms)
    if (norient == 2 && relaxed_ && !pairs.empty()) {
      neg_from_ = (int)(pairs.size() / 2);
      std::vector<int64_t> twice(pairs);
      twice.insert(twice.end(), pairs.begin(), pairs.end());
      pairs.swap(twice);
    }
    Pp_ = (int)(pairs.size() / 2);
    vals_.ensure(values_f.size());
    pairs_.ensure(std::max<size_t>(pairs.size(), 2));
    rck(hipMemcpy(vals_.p, values_f.data(), values_f.size() * sizeof(float), hipMemcpyHostToDevice), "cp");
    if (!pairs.empty())
      rck(hipMemcpy(pairs_.p, pairs.data(), pairs.size() * sizeof(int64_t), hipMemcpyHostToDevice), "cp");
    const size_t R = 2 * (size_t)batch_;
    rlo_.ensure(R * n0_); rhi_.ensure(R * n0_); rpart_.ensure(R);
    olb_.ensure(R); oub_.ensure(R); infeas_.ensure(R);
    Lc_.ensure(R * n0_); Uc_.ensure(R * n0_); L0_.ensure(R); Le_.ensure(R); U0_.ensure(R); Ue_.ensure(R);
    lay_lb_.ensure(R * net_.n_neurons); lay_ub_.ensure(R * net_.n_neurons);
    split_.ensure(2 * R); score_.ensure(2 * R);
    open_.ensure(batch_); choice_.ensure(batch_); idim_.ensure(batch_);
    cpts_.ensure(R * n0_); pe_lb_.ensure(R); pe_ub_.ensure(R);
    counters_.ensure(2);
    hcount_buf_.ensure(2 * sizeof(int));
    hcount_ = reinterpret_cast<int*>(hcount_buf_.p);
    // fp64 host copy of the network for the exact confirmation
    int np_ = 0;
    for (int l = 0; l < net_.n_layers; ++l) np_ = std::max(np_, net_.b_off[l] + net_.dims[l + 1]);
    std::vector<float> hf(np_);
    rck(hipMemcpy(hf.data(), flat_, np_ * sizeof(float), hipMemcpyDeviceToHost), "cp weights");
    exact_.n0 = n0_;
    exact_.n_layers = net_.n_layers;
    exact_.dims.assign(net_.dims, net_.dims + net_.n_layers + 1);
    exact_.w_off.assign(net_.w_off, net_.w_off + net_.n_layers);
    exact_.b_off.assign(net_.b_off, net_.b_off + net_.n_layers);
    exact_.w.assign(hf.begin(), hf.end());
    exact_.is_pa.assign(n0_, 0);
    exact_.is_ra.assign(n0_, 0);
    for (int k : pa_) exact_.is_pa[k] = 1;
    for (int k : ra_) exact_.is_ra[k] = 1;
    exact_.tau = tau_;
  }

  py::tuple solve(py::array_t<float, py::array::c_style | py::array::forcecast> lo,
                  py::array_t<float, py::array::c_style | py::array::forcecast> hi,
                  py::array_t<int8_t, py::array::c_style | py::array::forcecast> status0, int budget,
                  double time_budget, py::object confirm, uintptr_t stream_i) {
    hipStream_t st = (hipStream_t)stream_i;
    const auto t0 = std::chrono::steady_clock::now();
    const int P = (int)lo.shape(0);
    if (lo.ndim() != 2 || lo.shape(1) != n0_ || hi.shape(0) != P || status0.shape(0) != P)
      throw std::invalid_argument("relu solve: shape mismatch");
    box_lo_ = lo.data();
    box_hi_ = hi.data();
    status_.ensure(P);
    nodes_.ensure(P);
    nodes_start_.ensure(P);
    std::vector<int> run;
    for (int p = 0; p < P; ++p)
      if (status0.data()[p] == 3) run.push_back(p);
    const long long n_root = (long long)run.size() * Pp_;
    if (n_root > cap_) throw std::invalid_argument("more root nodes than pool capacity");
    ensure_pool(0, std::max<long long>(n_root, 1));
    // staged host block: status | part | pair | lo | hi (one H2D copy), then device memsets
    const int nbox = relaxed_ ? 4 : 2;     // lo, hi (+ relaxed: x' lo, hi)
    const size_t sb = (size_t)((P + 3) & ~3) + (size_t)n_root * (2 * sizeof(int) + nbox * n0_ * sizeof(float));
    hstage_.ensure(sb);
    {
      unsigned char* h = hstage_.p;
      std::memcpy(h, status0.data(), P);
      int* hp = reinterpret_cast<int*>(h + ((P + 3) & ~3));
      int* hq = hp + n_root;
      float* hl = reinterpret_cast<float*>(hq + n_root);
      float* hh = hl + n_root * n0_;
      float* hpl = hh + n_root * n0_;        // relaxed only
      float* hph = hpl + n_root * n0_;
      long long k = 0;
      for (int p : run)
        for (int q = 0; q < Pp_; ++q, ++k) {
          hp[k] = p;
          hq[k] = q;
          for (int d = 0; d < n0_; ++d) {
            hl[k * n0_ + d] = lo.data()[(size_t)p * n0_ + d];
            hh[k * n0_ + d] = hi.data()[(size_t)p * n0_ + d];
          }
          if (relaxed_) {                    // x': the RA dims widened by tau, unclipped
            for (int d = 0; d < n0_; ++d) {
              hpl[k * n0_ + d] = hl[k * n0_ + d];
              hph[k * n0_ + d] = hh[k * n0_ + d];
            }
            for (int d : ra_) {
              hpl[k * n0_ + d] -= tau_;
              hph[k * n0_ + d] += tau_;
            }
          }
        }
      stage_.ensure(sb);
      rck(hipMemcpyAsync(stage_.p, hstage_.p, sb, hipMemcpyHostToDevice, st), "cp stage");
      const unsigned char* d = stage_.p;
      rck(hipMemcpyAsync(status_.p, d, P, hipMemcpyDeviceToDevice, st), "cp status");
      d += (P + 3) & ~3;
      rck(hipMemcpyAsync(part_[0].p, d, n_root * sizeof(int), hipMemcpyDeviceToDevice, st), "cp part");
      d += n_root * sizeof(int);
      rck(hipMemcpyAsync(pair_[0].p, d, n_root * sizeof(int), hipMemcpyDeviceToDevice, st), "cp pair");
      d += n_root * sizeof(int);
      rck(hipMemcpyAsync(lo_[0].p, d, n_root * n0_ * sizeof(float), hipMemcpyDeviceToDevice, st), "cp lo");
      d += n_root * n0_ * sizeof(float);
      rck(hipMemcpyAsync(hi_[0].p, d, n_root * n0_ * sizeof(float), hipMemcpyDeviceToDevice, st), "cp hi");
      d += n_root * n0_ * sizeof(float);
      if (relaxed_) {
        rck(hipMemcpyAsync(plo_[0].p, d, n_root * n0_ * sizeof(float), hipMemcpyDeviceToDevice, st), "cp plo");
        d += n_root * n0_ * sizeof(float);
        rck(hipMemcpyAsync(phi_[0].p, d, n_root * n0_ * sizeof(float), hipMemcpyDeviceToDevice, st), "cp phi");
      }
      rck(hipMemsetAsync(phase_[0].p, 0, (size_t)n_root * 2 * nh_, st), "memset phase");
      rck(hipMemsetAsync(nodes_.p, 0, P * sizeof(int), st), "memset nodes");
      rck(hipMemsetAsync(nodes_start_.p, 0, P * sizeof(int), st), "memset nodes_start");
    }
    std::vector<int64_t> cex_x((size_t)P * n0_, 0), cex_xp((size_t)P * n0_, 0);
    std::vector<char> got(P, 0);
    int cur = 0;
    long long n_in = n_root;
    int levels = 0;
    bool timed_out = false;
    long long total = 0;
    {
      py::gil_scoped_release nogil;
      while (n_in > 0) {
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (el > time_budget) {
          timed_out = true;
          break;
        }
        const int nxt = cur ^ 1;
        ensure_pool(nxt, 2 * n_in);
        ensure_cand(n_in);
        rckl(fa_relu_reset_launch(counters_.p, st), "reset");
        for (long long s = 0; s < n_in; s += batch_) {
          const int nb = (int)std::min<long long>(batch_, n_in - s);
          level(cur, nxt, s, nb, P, budget, st);
        }
        rckl(fa_relu_settle_launch(P, status_.p, nodes_.p, nodes_start_.p, counters_.p, hcount_, st), "settle");
        rck(hipStreamSynchronize(st), "sync");
        total += n_in;
        ++levels;
        const int n_out = std::min((int)((volatile int*)hcount_)[0], pool_[nxt]);
        const int n_cand = std::min((int)((volatile int*)hcount_)[1], cand_alloc_);
        if (n_cand > 0) confirm_candidates(n_cand, confirm, got, cex_x, cex_xp, st);
        cur = nxt;
        n_in = n_out;
      }
    }
    // results
    const size_t hn_off = ((size_t)P + 15) & ~size_t(15);
    hout_.ensure(hn_off + (size_t)P * sizeof(int));
    rck(hipMemcpyAsync(hout_.p, status_.p, P, hipMemcpyDeviceToHost, st), "cp status out");
    rck(hipMemcpyAsync(hout_.p + hn_off, nodes_.p, P * sizeof(int), hipMemcpyDeviceToHost, st), "cp nodes out");
    rck(hipStreamSynchronize(st), "sync");
    const int8_t* hs = reinterpret_cast<const int8_t*>(hout_.p);
    const int* hn = reinterpret_cast<const int*>(hout_.p + hn_off);
    // partitions with nodes left after a time-out
    std::vector<char> left(P, 0);
    if (timed_out && n_in > 0) {
      std::vector<int> lp((size_t)n_in);
      rck(hipMemcpy(lp.data(), part_[cur].p, n_in * sizeof(int), hipMemcpyDeviceToHost), "cp left");
      for (int p : lp) left[p] = 1;
    }
    py::array_t<int8_t> status_out(P);
    py::array_t<int64_t> nodes_out(P);
    for (int p = 0; p < P; ++p) {
      int8_t v = hs[p];
      if (got[p]) v = 1;
      else if (v == 3 || v == 4) v = left[p] ? 0 : 2;     // every node closed => UNSAT
      status_out.mutable_data()[p] = v;
      nodes_out.mutable_data()[p] = hn[p];
    }
    py::array_t<int64_t> ax({P, n0_}), axp({P, n0_});
    std::memcpy(ax.mutable_data(), cex_x.data(), sizeof(int64_t) * cex_x.size());
    std::memcpy(axp.mutable_data(), cex_xp.data(), sizeof(int64_t) * cex_xp.size());
    py::dict stats;
    stats["levels"] = levels;
    stats["nodes"] = total;
    stats["timed_out"] = timed_out;
    stats["time"] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return py::make_tuple(status_out, ax, axp, nodes_out, stats);
  }

 private:
  void level(int cur, int nxt, long long s, int nb, int P, int budget, hipStream_t st) {
    ReluLevelArgs a{};
    a.Nn = nb; a.n0 = n0_; a.nh = nh_; a.npa = npa_;
    for (int k = 0; k < npa_; ++k) a.pa_idx[k] = pa_[k];
    a.pairs = pairs_.p; a.values = vals_.p; a.neg_from = neg_from_;
    a.part = part_[cur].p + s; a.pair = pair_[cur].p + s;
    a.xlo = lo_[cur].p + s * n0_; a.xhi = hi_[cur].p + s * n0_;
    a.phase = phase_[cur].p + s * 2 * nh_;
    a.rlo = rlo_.p; a.rhi = rhi_.p; a.rpart = rpart_.p;
    a.olb = olb_.p; a.oub = oub_.p; a.infeas = infeas_.p;
    a.Lc = Lc_.p; a.L0 = L0_.p; a.Le = Le_.p; a.Uc = Uc_.p; a.U0 = U0_.p; a.Ue = Ue_.p;
    a.split = split_.p;
    a.open = open_.p; a.choice = choice_.p; a.idim = idim_.p; a.cpts = cpts_.p;
    a.pe_lb = pe_lb_.p; a.pe_ub = pe_ub_.p;
    a.status = status_.p; a.part_nodes = nodes_.p; a.nodes_start = nodes_start_.p; a.budget = budget;
    a.opart = part_[nxt].p; a.opair = pair_[nxt].p; a.oxlo = lo_[nxt].p; a.oxhi = hi_[nxt].p;
    a.ophase = phase_[nxt].p; a.count_out = counters_.p; a.cap = pool_[nxt];
    a.cand_buf = reinterpret_cast<float*>(cand_host_.p); a.cand_count = counters_.p + 1; a.cand_cap = cand_alloc_;
    a.unit = (float)unit_;
    a.gmarg = rgamma(2 * n0_ + 4, unit_);
    if (relaxed_) {
      a.nra = (int)ra_.size();
      for (int k = 0; k < a.nra; ++k) a.ra_idx[k] = ra_[k];
      a.tau = tau_;
      a.xplo = plo_[cur].p + s * n0_; a.xphi = phi_[cur].p + s * n0_;
      a.oxplo = plo_[nxt].p; a.oxphi = phi_[nxt].p;
    }
    rckl(fa_relu_rows_launch(a, st), "relu rows");
    const int R = 2 * nb;
    rck(hipMemsetAsync(infeas_.p, 0, R, st), "memset infeas");
    BoundArgs b{};
    b.flat = flat_; b.lo = rlo_.p; b.hi = rhi_.p; b.R = R; b.symbolic = 1;
    b.out_lb = olb_.p; b.out_ub = oub_.p;
    b.Lc = Lc_.p; b.L0 = L0_.p; b.Le = Le_.p; b.Uc = Uc_.p; b.U0 = U0_.p; b.Ue = Ue_.p;
    b.layer_lb = lay_lb_.p; b.layer_ub = lay_ub_.p;
    b.V = 0;
    for (int k = 0; k < npa_; ++k) b.fold |= 1ull << pa_[k];
    b.skip_status = status_.p; b.skip_part = rpart_.p;
    b.phase_in = a.phase;           // node-major [n][2][nh] = row-major [2n + side][nh]
    b.infeas = infeas_.p;
    rckl(fa_bounds_launch(net_, b, st), "relu bounds");
    // hidden-layer bounds by back-substitution with the rows' fixed phases (refine.hip): tighter
    // relaxation intervals for the backward pass, and empty regions detected (infeas)
    if (refine_) {
      const int rc = fa_refine_launch(net_, b, st);
      if (rc == -1) refine_ = 0;
      else rckl(rc, "relu refine");
    }
    CrownPhaseArgs c{};
    c.flat = flat_; c.lo = rlo_.p; c.hi = rhi_.p; c.R = R; c.phase = a.phase;
    c.layer_lb = lay_lb_.p; c.layer_ub = lay_ub_.p; c.infeas = infeas_.p;
    c.out_lb = olb_.p; c.out_ub = oub_.p;
    c.Lc = Lc_.p; c.L0 = L0_.p; c.Le = Le_.p; c.Uc = Uc_.p; c.U0 = U0_.p; c.Ue = Ue_.p;
    c.split = split_.p; c.score = score_.p; c.low = nullptr;
    c.skip_status = status_.p; c.skip_part = rpart_.p;
    const int rc = fa_crown_phase_launch(net_, c, st);
    if (rc != 0) throw std::runtime_error("crown_phase launch failed, code " + std::to_string(rc));
    rckl(fa_relu_cert_launch(a, st), "relu cert");
    BoundArgs pb{};
    pb.flat = flat_; pb.lo = cpts_.p; pb.hi = cpts_.p; pb.R = R; pb.symbolic = 0;
    pb.out_lb = pe_lb_.p; pb.out_ub = pe_ub_.p;
    pb.row_open = open_.p; pb.open_mod = nb;
    // open_mod indexing of the point kernel: point r belongs to node r % open_mod; here points
    // 2n / 2n+1 belong to node n, so pass no skip (every pair is evaluated)
    pb.row_open = nullptr; pb.open_mod = 0;
    const int prc = fa_point_try_launch(net_, pb, st);
    if (prc < 0) rckl(-prc, "relu points");
    if (prc == 0) rckl(fa_bounds_launch(net_, pb, st), "relu points (bounds)");
    rckl(fa_relu_split_launch(a, st), "relu split");
  }

  void ensure_pool(int i, long long need) {
    const int want = (int)std::min<long long>(std::max<long long>(need, 1), cap_);
    if (want <= pool_[i]) return;
    int n = std::max(pool_[i], 1 << 14);
    while (n < want) n = (n > cap_ / 2) ? cap_ : n * 2;
    n = std::min(n, cap_);
    part_[i].ensure(n); pair_[i].ensure(n);
    lo_[i].ensure((size_t)n * n0_); hi_[i].ensure((size_t)n * n0_);
    if (relaxed_) { plo_[i].ensure((size_t)n * n0_); phi_[i].ensure((size_t)n * n0_); }
    phase_[i].ensure((size_t)n * 2 * nh_);
    pool_[i] = n;
  }

  void ensure_cand(long long need) {
    if (need <= cand_alloc_) return;
    long long n = std::max<long long>(cand_alloc_, 1 << 14);
    while (n < need) n *= 2;
    n = std::min<long long>(n, 1LL << 24);
    cand_host_.ensure((size_t)n * (2 * n0_ + 1) * sizeof(float));
    cand_alloc_ = (int)n;
  }

  // called WITHOUT the GIL; takes it only around the Python confirmation callback
  void confirm_candidates(int n_cand, py::object& confirm, std::vector<char>& got, std::vector<int64_t>& cex_x,
                          std::vector<int64_t>& cex_xp, hipStream_t st) {
    const size_t rec = (size_t)2 * n0_ + 1;
    // written by the split kernel into pinned host memory, retired by the level-end sync
    const float* hc = reinterpret_cast<const float*>(cand_host_.p);
    std::vector<float> buf((size_t)n_cand * 2 * n0_);
    std::vector<int> parts(n_cand);
    for (int i = 0; i < n_cand; ++i) {
      std::memcpy(buf.data() + (size_t)i * 2 * n0_, hc + (size_t)i * rec, sizeof(float) * 2 * n0_);
      std::memcpy(&parts[i], hc + (size_t)i * rec + 2 * n0_, sizeof(int));
    }
    std::vector<char> ok(n_cand, 0);
    std::vector<int> ask;
    for (int i = 0; i < n_cand; ++i) {
      const int r = exact_.check(buf.data() + (size_t)i * 2 * n0_, box_lo_ + (size_t)parts[i] * n0_,
                                 box_hi_ + (size_t)parts[i] * n0_);
      if (r < 0) ask.push_back(i);
      else ok[i] = (char)r;
    }
    if (!ask.empty()) {
      py::gil_scoped_acquire gil;
      const int na = (int)ask.size();
      py::array_t<float> abuf({na, 2 * n0_});
      py::array_t<int> aparts(na);
      for (int k = 0; k < na; ++k) {
        std::memcpy(abuf.mutable_data() + (size_t)k * 2 * n0_, buf.data() + (size_t)ask[k] * 2 * n0_,
                    sizeof(float) * 2 * n0_);
        aparts.mutable_data()[k] = parts[ask[k]];
      }
      py::array_t<bool> res = confirm(aparts, abuf).cast<py::array_t<bool>>();
      for (int k = 0; k < na; ++k) ok[ask[k]] = res.data()[k] ? 1 : 0;
    }
    std::vector<int> order(n_cand);
    for (int i = 0; i < n_cand; ++i) order[i] = i;
    const float* B = buf.data();
    const size_t w2 = (size_t)2 * n0_;
    std::sort(order.begin(), order.end(), [&](int x, int y) {
      if (parts[x] != parts[y]) return parts[x] < parts[y];
      return std::lexicographical_compare(B + x * w2, B + (x + 1) * w2, B + y * w2, B + (y + 1) * w2);
    });
    std::vector<int> newly;
    for (int i : order) {
      const int p = parts[i];
      if (!ok[i] || got[p]) continue;
      got[p] = 1;
      newly.push_back(p);
      for (int d = 0; d < n0_; ++d) {
        cex_x[(size_t)p * n0_ + d] = (int64_t)std::llround(B[(size_t)i * w2 + d]);
        cex_xp[(size_t)p * n0_ + d] = (int64_t)std::llround(B[(size_t)i * w2 + n0_ + d]);
      }
    }
    if (!newly.empty()) {
      // SAT partitions stop: their nodes are skipped from the next level on (status filter)
      idx_.ensure(newly.size());
      hidx_.ensure(newly.size() * sizeof(int));
      std::memcpy(hidx_.p, newly.data(), newly.size() * sizeof(int));
      rck(hipMemcpyAsync(idx_.p, hidx_.p, newly.size() * sizeof(int), hipMemcpyHostToDevice, st), "cp idx");
      // status 1 (SAT) for each: a tiny host loop of memsets keeps this file free of extra kernels
      for (size_t k = 0; k < newly.size(); ++k)
        rck(hipMemsetAsync(status_.p + newly[k], 1, 1, st), "set sat");
      rck(hipStreamSynchronize(st), "sync");
    }
  }

  NetDesc net_;
  const float* flat_;
  std::vector<int> pa_;
  int cap_, batch_;
  double unit_;
  int refine_ = 0;          // phase-aware back-substituted hidden-layer bounds (ReluConfig.refine)
  std::vector<int> ra_;     // relaxed queries: RA dims and tolerance (x' box per node)
  float tau_ = 0.f;
  bool relaxed_ = false;
  int n0_ = 0, nh_ = 0, npa_ = 0, V_ = 0, Pp_ = 0;
  int neg_from_ = 0;        // > 0: pairs [neg_from_, Pp_) are the reverse orientation
  int pool_[2] = {0, 0};
  int cand_alloc_ = 0;
  fa_exact::ExactChecker exact_;
  const float* box_lo_ = nullptr;
  const float* box_hi_ = nullptr;
  RBuf<float> vals_;
  RBuf<int64_t> pairs_;
  RBuf<int> part_[2], pair_[2];
  RBuf<float> lo_[2], hi_[2], plo_[2], phi_[2];
  RBuf<int8_t> phase_[2];
  RBuf<float> rlo_, rhi_, olb_, oub_, Lc_, Uc_, L0_, Le_, U0_, Ue_, lay_lb_, lay_ub_, score_, cpts_, pe_lb_, pe_ub_;
  RBuf<int> rpart_, split_, choice_, idim_, counters_, nodes_, nodes_start_, idx_;
  RBuf<uint8_t> infeas_, open_;
  RBuf<int8_t> status_;
  RBuf<unsigned char> stage_;
  fa_mem::HostBuf hcount_buf_{true};   // coherent: the settle kernel writes the level counters
  int* hcount_ = nullptr;
  // pinned staging; same buffer-lifetime rule as BabRuntime (released / regrown only after the
  // stream synchronisation that retires its last copy)
  fa_mem::HostBuf hstage_, hout_, hidx_;
  fa_mem::HostBuf cand_host_{true};   // candidate records (coherent pinned, written by the split kernel)
};

void register_relu(py::module& m) {
  py::class_<ReluRuntime>(m, "ReluRuntime")
      .def(py::init<py::handle, uintptr_t, std::vector<int>, std::vector<float>, std::vector<int64_t>, int, int,
                    double, int, std::vector<int>, double, int>(),
           py::arg("net"), py::arg("flat"), py::arg("pa"), py::arg("values_f"), py::arg("pairs"),
           py::arg("capacity"), py::arg("batch_nodes"), py::arg("unit"), py::arg("refine") = 0,
           py::arg("ra") = std::vector<int>(), py::arg("tau") = 0.0, py::arg("norient") = 1)
      .def("solve", &ReluRuntime::solve, py::arg("lo"), py::arg("hi"), py::arg("status"), py::arg("budget"),
           py::arg("time_budget"), py::arg("confirm"), py::arg("stream"));
}
