// Native branch-and-bound driver (C++ host runtime around the HIP kernels).
//
// The reference decides each partition with one Z3 check() (src/AC/Verify-AC.py:127-163).  Here
// all partitions of a chunk are decided together by a breadth-first branch-and-bound whose node
// pool lives in device memory.  One BFS level = ceil(frontier / batch) sub-batches of
//   bounds (symbolic, node-row expansion)  [+ bounds on x' boxes for relaxed queries]
//   certify (pair LP certificate + pick)   -> open / leaf / split scores / candidate pair
//   bounds (interval, candidate points)    -> rigorous point evaluation of the candidates
//   split                                  -> children in the other pool, candidates flagged
// followed by ONE host synchronisation (two counters).  Flagged candidates are confirmed
// exactly by a Python callback (rational/fp64 check of the exact network); confirmed partitions
// flip to SAT on the device.  Partitions whose nodes are all closed end UNSAT; budgets and the
// time limit end the rest UNKNOWN.  The branching factor per level (2^m) grows when the
// frontier is small so that tail levels still fill the GPU.
#include <hip/hip_runtime.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <utility>
#include <vector>

#include "args.h"
#include "devmem.h"
#include "exact_host.h"

namespace py = pybind11;

#define FA_CAND_MAX (1LL << 24)   // candidates confirmable per BFS level

extern "C" int fa_bounds_launch(const NetDesc& net, BoundArgs args, hipStream_t stream);
extern "C" int fa_point_try_launch(const NetDesc& net, BoundArgs a, hipStream_t stream);
extern "C" int fa_certify_launch(CertArgs a, hipStream_t stream);
extern "C" int fa_split_launch(SplitArgs a, hipStream_t stream);
extern "C" int fa_mark_unknown_launch(const int* part, int n, int8_t* status, hipStream_t stream);
extern "C" int fa_set_status_launch(const int* idx, int n, int8_t* status, int8_t v, hipStream_t stream);
extern "C" int fa_settle_launch(SettleArgs s, hipStream_t stream);
extern "C" int fa_crown_launch(const NetDesc& net, BoundArgs a, hipStream_t stream);
extern "C" int fa_refine_launch(const NetDesc& net, BoundArgs a, hipStream_t stream);
extern "C" int fa_backward_launch(const NetDesc& net, BoundArgs a, hipStream_t stream);
extern "C" int fa_refine_crown_launch(const NetDesc& net, BoundArgs a, hipStream_t stream);
extern "C" int fa_bab_init_launch(BabInitArgs a, hipStream_t stream);
extern "C" int fa_bab_finish_launch(int P, const int8_t* status, const int* nodes, const int* open_left, int* out,
                                    hipStream_t stream);

// defined in bindings.cpp
const NetDesc& fa_net_desc(py::handle net);

namespace {

void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
void ckl(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string(what) + " launch failed, code " + std::to_string(rc));
}

using fa_mem::DevBuf;

// A/B switch of the closed-node skip in the candidate point kernel (FAIRIFY_POINT_SKIP_CLOSED=0: off)
bool point_skip_closed() {
  static const bool v = [] {
    const char* e = getenv("FAIRIFY_POINT_SKIP_CLOSED");
    return !(e && e[0] == '0');
  }();
  return v;
}

// A/B switch of the closed-node early-out in the pair certificate (FAIRIFY_CERT_SKIP_CLOSED=0: off)
bool cert_skip_closed() {
  static const bool v = [] {
    const char* e = getenv("FAIRIFY_CERT_SKIP_CLOSED");
    return !(e && e[0] == '0');
  }();
  return v;
}

// A/B switch of the level end fused into the last split launch (FAIRIFY_FUSE_SETTLE=1: fused;
// default its own launch -- BaBConfig.fuse_settle sets it per solve)
bool fuse_settle() {
  static const bool v = [] {
    const char* e = getenv("FAIRIFY_FUSE_SETTLE");
    return e && e[0] == '1';
  }();
  return v;
}

// A/B switch: refine skips nodes its forward bounds already close (FAIRIFY_REFINE_SKIP_SIGNDEF=0: off)
bool skip_signdef() {
  static const bool v = [] {
    const char* e = getenv("FAIRIFY_REFINE_SKIP_SIGNDEF");
    return !(e && e[0] == '0');
  }();
  return v;
}

float gamma_up(int k, double unit) {
  const double ku = (k + 2) * unit;
  return std::nextafter((float)(ku / (1.0 - ku)), INFINITY);
}

}  // namespace

class BabRuntime {
 public:
  BabRuntime(py::handle net, uintptr_t flat, std::vector<int> pa, std::vector<float> values_f,
             std::vector<int64_t> values_i, std::vector<int64_t> pairs, std::vector<int> ra, float tau,
             std::vector<uint8_t> shared, int capacity, int batch_nodes, int cand_cap, double unit, bool crown,
             int split_target, int refine, bool smear)
      : net_(fa_net_desc(net)),
        flat_((const float*)flat),
        pa_(std::move(pa)),
        ra_(std::move(ra)),
        tau_(tau),
        cap_(capacity),
        batch_(batch_nodes),
        cand_cap_(cand_cap),
        unit_(unit),
        crown_(crown),
        refine_(crown ? refine : 0),
        smear_(smear),
        split_target_(std::max(2, split_target)) {
    n0_ = net_.dims[0];
    npa_ = (int)pa_.size();
    if (npa_ == 0 || npa_ > FA_CMAX_PA || (int)ra_.size() > FA_MAX_RA) throw std::invalid_argument("bad PA/RA");
    V_ = (int)(values_i.size() / npa_);
    Pp_ = (int)(pairs.size() / 2);
    relaxed_ = !ra_.empty() && tau_ > 0;
    norient_ = relaxed_ ? 2 : 1;
    if ((int)shared.size() != n0_) throw std::invalid_argument("shared mask size");
    vals_f_.ensure(values_f.size());
    vals_i_.ensure(values_i.size());
    pairs_.ensure(pairs.size());
    shared_.ensure(shared.size());
    ck(hipMemcpy(vals_f_.p, values_f.data(), values_f.size() * sizeof(float), hipMemcpyHostToDevice), "cp");
    ck(hipMemcpy(vals_i_.p, values_i.data(), values_i.size() * sizeof(int64_t), hipMemcpyHostToDevice), "cp");
    ck(hipMemcpy(pairs_.p, pairs.data(), pairs.size() * sizeof(int64_t), hipMemcpyHostToDevice), "cp");
    ck(hipMemcpy(shared_.p, shared.data(), shared.size(), hipMemcpyHostToDevice), "cp");
    // node pools grow on demand (geometrically) up to cap_ = the configured maximum
    pool_[0] = pool_[1] = 0;
    const size_t R = (size_t)batch_ * V_;
    for (int s = 0; s < (relaxed_ ? 2 : 1); ++s) {
      Lc_[s].ensure(R * n0_);
      Uc_[s].ensure(R * n0_);
      L0_[s].ensure(R); Le_[s].ensure(R); U0_[s].ensure(R); Ue_[s].ensure(R);
      olb_[s].ensure(R); oub_[s].ensure(R);
      if (crown_ || smear_) {
        lay_lb_[s].ensure(R * net_.n_neurons);
        lay_ub_[s].ensure(R * net_.n_neurons);
      }
    }
    const size_t Q = (size_t)Pp_ * norient_;
    gmin_.ensure(batch_ * Q);
    tstar_.ensure(batch_ * Q);
    open_.ensure(batch_);
    leaf_.ensure(batch_);
    score_.ensure(batch_);
    split_.ensure(batch_);
    cv_.ensure(batch_);
    co_.ensure(batch_);
    cand_.ensure((size_t)2 * batch_ * n0_);
    scores_.ensure((size_t)batch_ * 2 * n0_);
    pe_lb_.ensure(2 * (size_t)batch_);
    pe_ub_.ensure(2 * (size_t)batch_);
    ensure_cand(cand_cap_);
    counters_.ensure(5);   // two slots of (children, candidates), alternating per level, + the
                           // fused settle's workgroup counter
    // fine-grained (coherent) pinned words: the settle kernel writes the level counters here
    hcount_buf_.ensure(2 * sizeof(int));
    hcount_ = reinterpret_cast<int*>(hcount_buf_.p);
    // host fp64 copy of [W_0|b_0|W_1|b_1|...] for the native exact confirmation
    int np_ = 0;
    for (int l = 0; l < net_.n_layers; ++l) np_ = std::max(np_, net_.b_off[l] + net_.dims[l + 1]);
    std::vector<float> hf(np_);
    ck(hipMemcpy(hf.data(), flat_, np_ * sizeof(float), hipMemcpyDeviceToHost), "cp weights");
    exact_.n0 = n0_;
    exact_.n_layers = net_.n_layers;
    exact_.dims.assign(net_.dims, net_.dims + net_.n_layers + 1);
    exact_.w_off.assign(net_.w_off, net_.w_off + net_.n_layers);
    exact_.b_off.assign(net_.b_off, net_.b_off + net_.n_layers);
    exact_.w.assign(hf.begin(), hf.end());
    exact_.is_pa.assign(n0_, 0);
    exact_.is_ra.assign(n0_, 0);
    for (int k : pa_) exact_.is_pa[k] = 1;
    if (relaxed_)
      for (int k : ra_) exact_.is_ra[k] = 1;
    exact_.tau = tau_;
    // |W0| transposed for the smear split scores: row j = neuron j's |W0[:, j]|, zero padded to the
    // certify kernel's register width NM (16 or 32 input dims), so a neuron is NM/4 float4 loads
    if (smear_ && n0_ > 32) smear_ = false;
    if (smear_) {
      const int nm = n0_ <= 16 ? 16 : 32, n1 = net_.dims[1];
      std::vector<float> wt((size_t)n1 * nm, 0.f);
      for (int j = 0; j < n1; ++j)
        for (int i = 0; i < n0_; ++i) wt[(size_t)j * nm + i] = std::fabs(hf[(size_t)net_.w_off[0] + (size_t)i * n1 + j]);
      w0t_.ensure(wt.size());
      ck(hipMemcpy(w0t_.p, wt.data(), wt.size() * sizeof(float), hipMemcpyHostToDevice), "cp w0t");
    }
  }

  void set_fuse_settle(bool v) { fuse_settle_ = v; }

  py::tuple solve(py::array_t<float, py::array::c_style | py::array::forcecast> lo,
                  py::array_t<float, py::array::c_style | py::array::forcecast> hi,
                  py::array_t<int8_t, py::array::c_style | py::array::forcecast> status0, int budget,
                  double time_budget, uintptr_t dead_part, py::object confirm, uintptr_t stream_i,
                  bool native_exact, int budget2, int max_w, std::vector<std::pair<int, int>> esc_steps) {
    const bool inline_esc = budget2 > budget && max_w > 0;
    // intermediate escalation steps strictly between budget and budget2, increasing budgets
    EscSteps esc{};
    for (const auto& bo : esc_steps)
      if (bo.first > (esc.n ? esc.budget[esc.n - 1] : budget) && bo.first < budget2 && esc.n < FA_MAX_ESC) {
        esc.budget[esc.n] = bo.first;
        esc.open[esc.n] = bo.second;
        ++esc.n;
      }
    hipStream_t st = (hipStream_t)stream_i;
    native_exact_ = native_exact;
    box_lo_ = lo.data();
    box_hi_ = hi.data();
    const auto t0 = std::chrono::steady_clock::now();
    const int P = (int)lo.shape(0);
    if (lo.ndim() != 2 || lo.shape(1) != n0_ || hi.shape(0) != P || status0.shape(0) != P)
      throw std::invalid_argument("solve: shape mismatch");
    status_.ensure(P);
    nodes_.ensure(P);
    open_left_.ensure(P);
    lvl_open_.ensure(P);
    nodes_start_.ensure(P);
    prev_start_.ensure(P);
    if (inline_esc) {
      pbudget_.ensure(P);
      prob_.ensure(P);
    }
    int slot = 0;
    // initial pool: running partitions.  Everything the device needs at the start goes through
    // ONE pinned staging block + one H2D copy + one init kernel (status, per-partition state,
    // root boxes, counters) instead of four copies and six memsets.
    const int8_t* hstatus = status0.data();
    std::vector<int> run;
    for (int p = 0; p < P; ++p)
      if (hstatus[p] == 3) run.push_back(p);
    if ((int)run.size() > cap_) throw std::invalid_argument("more partitions than pool capacity");
    ensure_pool(0, std::max<long long>((long long)run.size(), 1));
    const size_t nrun = run.size();
    const size_t st_bytes = (size_t)((P + 3) & ~3) + nrun * sizeof(int) + 2 * nrun * n0_ * sizeof(float);
    hstage_.ensure(st_bytes);
    stage_.ensure(st_bytes);
    {
      unsigned char* h = hstage_.p;
      std::memcpy(h, hstatus, P);
      int* hr = reinterpret_cast<int*>(h + ((P + 3) & ~3));
      std::memcpy(hr, run.data(), nrun * sizeof(int));
      float* hl = reinterpret_cast<float*>(hr + nrun);
      float* hh = hl + nrun * n0_;
      for (size_t i = 0; i < nrun; ++i)
        for (int d = 0; d < n0_; ++d) {
          hl[i * n0_ + d] = lo.data()[(size_t)run[i] * n0_ + d];
          hh[i * n0_ + d] = hi.data()[(size_t)run[i] * n0_ + d];
        }
    }
    ck(hipMemcpyAsync(stage_.p, hstage_.p, st_bytes, hipMemcpyHostToDevice, st), "cp stage");
    {
      BabInitArgs ia{};
      ia.P = P; ia.n_run = (int)nrun; ia.n0 = n0_;
      ia.stage = stage_.p;
      ia.status = status_.p; ia.nodes = nodes_.p; ia.open_left = open_left_.p; ia.lvl_open = lvl_open_.p;
      ia.nodes_start = nodes_start_.p; ia.prev_start = prev_start_.p;
      ia.part = part_[0].p; ia.xlo = lo_[0].p; ia.xhi = hi_[0].p;
      ia.xplo = relaxed_ ? plo_[0].p : nullptr; ia.xphi = relaxed_ ? phi_[0].p : nullptr;
      ia.nra = relaxed_ ? (int)ra_.size() : 0;
      for (int k = 0; k < ia.nra; ++k) ia.ra_idx[k] = ra_[k];
      ia.tau = tau_;
      ia.counters = counters_.p;
      ia.pbudget = inline_esc ? pbudget_.p : nullptr;
      ia.prob = inline_esc ? prob_.p : nullptr;
      ia.budget = budget;
      ckl(fa_bab_init_launch(ia, st), "bab_init");
    }
    int cur = 0;
    int n_in = (int)nrun;
    // host result buffers
    std::vector<int64_t> cex_x((size_t)P * n0_, 0), cex_xp((size_t)P * n0_, 0);
    std::vector<char> got(P, 0);
    int levels = 0, launches = 0, cand_overflow = 0;
    long long total_nodes = 0;
    bool timed_out = false;
    {
    // the level loop runs without the GIL: several models/streams can be driven from Python threads
    py::gil_scoped_release nogil;
    while (n_in > 0) {
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > time_budget) {
        ckl(fa_mark_unknown_launch(part_[cur].p, n_in, status_.p, st), "mark");
        timed_out = true;
        break;
      }
      int* cnt = counters_.p + 2 * slot;
      const int nxt = cur ^ 1;
      // every kernel of the previous level has finished (level-end sync), so the next pool
      // can be re-allocated safely.  Per partition with w nodes in the level the branching rule
      // makes at most max(split_target, 2 w) children: <= 2 n_in + split_target * min(P, n_in)
      ensure_pool(nxt, 2LL * n_in + (long long)split_target_ * std::min(P, n_in));
      // candidate buffer for the whole level (one per inner node, every PA pair of a leaf): a
      // capped buffer would drop candidates depending on which partitions share the chunk
      ensure_cand(std::min<long long>((long long)n_in * std::max(1, Pp_ * norient_), FA_CAND_MAX));
      // level end: its own launch, or (fuse_settle_) fused into the level's last split launch
      // whose last workgroup settles
      SettleArgs se{};
      se.P = P; se.status = status_.p; se.lvl_open = lvl_open_.p; se.part_open = open_left_.p;
      se.part_nodes = nodes_.p; se.nodes_start = nodes_start_.p; se.prev_start = prev_start_.p;
      se.counters_cur = cnt; se.counters_next = counters_.p + 2 * (slot ^ 1); se.host_counts = hcount_;
      se.pbudget = inline_esc ? pbudget_.p : nullptr; se.prob = inline_esc ? prob_.p : nullptr;
      se.budget2 = budget2; se.max_open = max_w; se.esc = esc;
      se.done = counters_.p + 4;
      bool settled = false;
      for (int s = 0; s < n_in; s += batch_) {
        const int nb = std::min(batch_, n_in - s);
        const float* blo = lo_[cur].p + (size_t)s * n0_;
        const float* bhi = hi_[cur].p + (size_t)s * n0_;
        const float* bplo = relaxed_ ? plo_[cur].p + (size_t)s * n0_ : blo;
        const float* bphi = relaxed_ ? phi_[cur].p + (size_t)s * n0_ : bhi;
        const int* bpart = part_[cur].p + s;
        launch_bounds(blo, bhi, bpart, nb, 0, dead_part, st);
        if (relaxed_) launch_bounds(bplo, bphi, bpart, nb, 1, dead_part, st);
        const int sx = relaxed_ ? 1 : 0;
        CertArgs c{};
        c.Nn = nb; c.n0 = n0_; c.V = V_; c.Pp = Pp_; c.norient = norient_;
        c.Lc = Lc_[0].p; c.L0 = L0_[0].p; c.Le = Le_[0].p; c.Uc = Uc_[0].p; c.U0 = U0_[0].p; c.Ue = Ue_[0].p;
        c.Lcp = Lc_[sx].p; c.L0p = L0_[sx].p; c.Lep = Le_[sx].p;
        c.Ucp = Uc_[sx].p; c.U0p = U0_[sx].p; c.Uep = Ue_[sx].p;
        c.olb = olb_[0].p; c.oub = oub_[0].p; c.olbp = olb_[sx].p; c.oubp = oub_[sx].p;
        c.xlo = blo; c.xhi = bhi; c.xplo = bplo; c.xphi = bphi;
        c.pairs = pairs_.p; c.values = vals_i_.p; c.npa = npa_;
        for (int k = 0; k < npa_; ++k) c.pa_idx[k] = pa_[k];
        c.nra = relaxed_ ? (int)ra_.size() : 0;
        for (int k = 0; k < c.nra; ++k) c.ra_idx[k] = ra_[k];
        c.tau = tau_;
        c.shared = shared_.p;
        c.unit = (float)unit_;
        c.gmarg = gamma_up(2 * n0_ + 4, unit_);
        c.gmin = gmin_.p; c.tstar = tstar_.p;
        c.open = open_.p; c.score = score_.p; c.split_dim = split_.p;
        c.cand_x = cand_.p; c.cand_xp = cand_.p + (size_t)nb * n0_;
        c.cand_v = cv_.p; c.cand_o = co_.p;
        c.scores = scores_.p; c.leaf = leaf_.p;
        if (cert_skip_closed()) { c.skip_closed = 1; c.status = status_.p; c.part = bpart; }
        if (smear_ && !relaxed_) {
          c.smear = 1;
          c.lay_lb = lay_lb_[0].p; c.lay_ub = lay_ub_[0].p; c.lay_N = net_.n_neurons;
          c.W0T = w0t_.p; c.n1 = net_.dims[1];
        }
        ckl(fa_certify_launch(c, st), "certify");
        // rigorous interval evaluation of the candidate pairs (rows: x then x')
        BoundArgs b{};
        b.flat = flat_; b.lo = cand_.p; b.hi = cand_.p; b.R = 2 * nb; b.symbolic = 0;
        b.out_lb = pe_lb_.p; b.out_ub = pe_ub_.p;
        // per-point partition ids only matter for the heuristic (masked) nets: points k and
        // nb + k (x and x' of node k) both read bpart[k]
        if (dead_part) { b.node_part = bpart; b.part_mod = nb; b.dead_part = (const uint8_t*)dead_part; }
        if (point_skip_closed()) { b.row_open = open_.p; b.open_mod = nb; }
        const int prc = fa_point_try_launch(net_, b, st);
        if (prc < 0) ckl(-prc, "points");
        if (prc == 0) ckl(fa_bounds_launch(net_, b, st), "bounds(points)");
        SplitArgs sa{};
        sa.Nn = nb; sa.n0 = n0_; sa.relaxed = relaxed_ ? 1 : 0; sa.nra = relaxed_ ? (int)ra_.size() : 0;
        for (int k = 0; k < sa.nra; ++k) sa.ra_idx[k] = ra_[k];
        sa.V = V_; sa.Pp = Pp_; sa.norient = norient_; sa.tau = tau_;
        sa.xlo = blo; sa.xhi = bhi; sa.xplo = bplo; sa.xphi = bphi; sa.part = bpart;
        sa.open = open_.p; sa.leaf = leaf_.p; sa.scores = scores_.p;
        sa.cand_x = c.cand_x; sa.cand_xp = c.cand_xp; sa.pe_lb = pe_lb_.p; sa.pe_ub = pe_ub_.p;
        sa.olb = c.olb; sa.oub = c.oub; sa.olbp = c.olbp; sa.oubp = c.oubp;
        sa.pairs = pairs_.p; sa.values = vals_i_.p; sa.npa = npa_;
        for (int k = 0; k < npa_; ++k) sa.pa_idx[k] = pa_[k];
        sa.shared = shared_.p;
        sa.status = status_.p; sa.part_nodes = nodes_.p; sa.part_open = open_left_.p; sa.lvl_open = lvl_open_.p;
        sa.nodes_start = nodes_start_.p;
        sa.prev_start = prev_start_.p;
        sa.budget = budget; sa.m = FA_MAX_SPLIT; sa.target = split_target_;
        sa.pbudget = inline_esc ? pbudget_.p : nullptr;
        sa.prob = inline_esc ? prob_.p : nullptr;
        sa.budget2 = budget2;
        sa.oxlo = lo_[nxt].p; sa.oxhi = hi_[nxt].p;
        sa.oxplo = relaxed_ ? plo_[nxt].p : nullptr; sa.oxphi = relaxed_ ? phi_[nxt].p : nullptr;
        sa.opart = part_[nxt].p; sa.count_out = cnt; sa.cap = pool_[nxt];
        sa.cand_buf = reinterpret_cast<float*>(cand_host_.p); sa.cand_count = cnt + 1;
        sa.cand_cap = cand_alloc_;
        if (s + nb >= n_in && fuse_settle_) {
          sa.settle = se;
          settled = true;
        }
        ckl(fa_split_launch(sa, st), "split");
        launches += (relaxed_ ? 2 : 1) * (refine_ == 2 ? 1 : 2) + 3;   // bounding launches + certify, points, split
      }
      if (!settled) {
        ckl(fa_settle_launch(se, st), "settle");
        ++launches;
      }
      ck(hipStreamSynchronize(st), "sync");
      slot ^= 1;
      total_nodes += n_in;
      const int n_out = std::min((int)((volatile int*)hcount_)[0], pool_[nxt]);
      const int n_cand_all = ((volatile int*)hcount_)[1];
      const int n_cand = std::min(n_cand_all, cand_alloc_);
      if (n_cand_all > cand_alloc_) ++cand_overflow;
      ++levels;
      if (n_cand > 0) confirm_candidates(n_cand, confirm, got, cex_x, cex_xp, st);
      cur = nxt;
      n_in = n_out;
    }
    }
    // results: one pack kernel + one D2H copy into pinned memory
    out_.ensure((size_t)3 * P);
    hout_.ensure((size_t)3 * P * sizeof(int));
    ckl(fa_bab_finish_launch(P, status_.p, nodes_.p, open_left_.p, out_.p, st), "bab_finish");
    ck(hipMemcpyAsync(hout_.p, out_.p, (size_t)3 * P * sizeof(int), hipMemcpyDeviceToHost, st), "cp out");
    ck(hipStreamSynchronize(st), "sync");
    const int* hres = reinterpret_cast<const int*>(hout_.p);
    py::array_t<int8_t> status_out(P);
    py::array_t<int64_t> nodes_out(P), open_out(P);
    for (int p = 0; p < P; ++p) {
      int8_t v = (int8_t)hres[p];
      if (got[p]) v = 1;
      else if (v == 3) v = timed_out ? 0 : 2;   // all nodes closed => UNSAT
      status_out.mutable_data()[p] = v;
      nodes_out.mutable_data()[p] = hres[P + p];
      open_out.mutable_data()[p] = (v == 0) ? hres[2 * P + p] : 0;
    }
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    py::dict stats;
    stats["levels"] = levels;
    stats["launches"] = launches;
    stats["cand_overflow_levels"] = cand_overflow;
    stats["nodes"] = total_nodes;
    stats["time"] = el;
    stats["timed_out"] = timed_out;
    py::array_t<int64_t> ax({P, n0_}), axp({P, n0_});
    std::memcpy(ax.mutable_data(), cex_x.data(), sizeof(int64_t) * cex_x.size());
    std::memcpy(axp.mutable_data(), cex_xp.data(), sizeof(int64_t) * cex_xp.size());
    stats["open_left"] = open_out;
    return py::make_tuple(status_out, ax, axp, nodes_out, stats);
  }

 private:
  void launch_bounds(const float* lo, const float* hi, const int* part, int nb, int slot, uintptr_t dead_part,
                     hipStream_t st) {
    BoundArgs b{};
    b.flat = flat_;
    b.lo = lo;
    b.hi = hi;
    b.R = nb * V_;
    b.symbolic = 1;
    b.out_lb = olb_[slot].p; b.out_ub = oub_[slot].p;
    b.Lc = Lc_[slot].p; b.L0 = L0_[slot].p; b.Le = Le_[slot].p;
    b.Uc = Uc_[slot].p; b.U0 = U0_[slot].p; b.Ue = Ue_[slot].p;
    b.V = V_;
    b.npa = npa_;
    for (int k = 0; k < npa_; ++k) b.pa_idx[k] = pa_[k];
    b.values = vals_f_.p;
    if (dead_part) {
      b.node_part = part;
      b.dead_part = (const uint8_t*)dead_part;
    }
    b.skip_status = status_.p;     // skip nodes of partitions decided / stopped earlier
    b.skip_part = part;
    if (refine_ == 2) {
      // backward-only bounding (refine.hip mode FULL): one launch computes every hidden layer's
      // bounds and the logit's forms, no forward pass and no output pass; -1: the network does not
      // fit, fall back to forward + refine + output pass (layer bounds written only for the smear
      // split scores)
      if (smear_) { b.layer_lb = lay_lb_[slot].p; b.layer_ub = lay_ub_[slot].p; }
      const int rc = fa_backward_launch(net_, b, st);
      if (rc == 0) return;
      if (rc != -1) ckl(rc, "backward");
      refine_ = 1;
    }
    if (crown_ || smear_) {
      b.layer_lb = lay_lb_[slot].p;
      b.layer_ub = lay_ub_[slot].p;
    }
    ckl(fa_bounds_launch(net_, b, st), "bounds");
    // hidden-layer bounds tightened by back-substitution (refine.hip) before the output pass uses
    // them as relaxation intervals; a network the kernel cannot hold (-1) keeps the forward bounds
    if (refine_ == 1) {
      // refined hidden-layer bounds and the logit's backward pass in one launch; nodes whose
      // forward bounds already exclude every ordered pair (single PA: Pp = V (V - 1)) are skipped
      b.skip_signdef = (!relaxed_ && npa_ == 1 && Pp_ == V_ * (V_ - 1) && skip_signdef()) ? 1 : 0;
      const int rc = fa_refine_crown_launch(net_, b, st);
      if (rc == 0) return;
      if (rc != -1) ckl(rc, "refine");
      refine_ = 0;
    }
    // backward output bounds: tighter forms / logit bounds for the certificate.  A network the
    // kernel cannot hold (layer > 256 wide or weights beyond the LDS budget: -1) keeps the
    // forward forms, which are sound on their own.
    if (crown_) {
      const int rc = fa_crown_launch(net_, b, st);
      if (rc == -1) crown_ = false;
      else ckl(rc, "crown");
    }
  }

  // grow pool `i` to hold at least `need` nodes (clamped to cap_; over-capacity children make
  // their partition UNKNOWN in the split kernel, which stays sound)
  void ensure_pool(int i, long long need) {
    const int want = (int)std::min<long long>(std::max<long long>(need, 1), cap_);
    if (want <= pool_[i]) return;
    int n = std::max(pool_[i], 1 << 16);
    while (n < want) n = (n > cap_ / 2) ? cap_ : n * 2;
    n = std::min(n, cap_);
    const size_t cn = (size_t)n * n0_;
    lo_[i].ensure(cn);
    hi_[i].ensure(cn);
    part_[i].ensure(n);
    if (relaxed_) {
      plo_[i].ensure(cn);
      phi_[i].ensure(cn);
    }
    pool_[i] = n;
  }

  void ensure_cand(long long need) {
    if (need <= cand_alloc_) return;
    long long n = std::max<long long>(cand_alloc_, 1 << 16);
    while (n < need) n *= 2;
    n = std::min<long long>(n, FA_CAND_MAX);
    cand_host_.ensure((size_t)n * (2 * n0_ + 1) * sizeof(float));
    cand_alloc_ = (int)n;
  }

  // called WITHOUT the GIL; takes it only around the Python confirmation callback
  void confirm_candidates(int n_cand, py::object& confirm, std::vector<char>& got, std::vector<int64_t>& cex_x,
                          std::vector<int64_t>& cex_xp, hipStream_t st) {
    const size_t rec = (size_t)2 * n0_ + 1;             // x, x', partition id (int bits)
    // the split kernel wrote the records straight into pinned host memory, and the level-end
    // synchronisation retired it: no copy, no second round trip per level
    std::vector<float> buf((size_t)n_cand * 2 * n0_);
    std::vector<int> parts(n_cand);
    {
      const float* hc = reinterpret_cast<const float*>(cand_host_.p);
      for (int i = 0; i < n_cand; ++i) {
        std::memcpy(buf.data() + (size_t)i * 2 * n0_, hc + (size_t)i * rec, sizeof(float) * 2 * n0_);
        std::memcpy(&parts[i], hc + (size_t)i * rec + 2 * n0_, sizeof(int));
      }
    }
    std::vector<char> ok(n_cand, 0);
    // native exact check (no GIL): pair constraints + fp64 logits with a rigorous rounding
    // bound; only pairs whose sign the bound cannot settle go to the Python callback
    // (exact rational arithmetic), as do all pairs of per-partition (masked) networks
    std::vector<int> ask;
    if (native_exact_) {
      for (int i = 0; i < n_cand; ++i) {
        const int r = exact_check(buf.data() + (size_t)i * 2 * n0_, parts[i]);
        if (r < 0) ask.push_back(i);
        else ok[i] = (char)r;
      }
    } else {
      ask.resize(n_cand);
      for (int i = 0; i < n_cand; ++i) ask[i] = i;
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
    // the device appended candidates in atomic order: pick each partition's witness by a fixed
    // order (partition, then the pair lexicographically) so the reported pair does not depend
    // on scheduling
    std::vector<int> newly;
    const float* B = buf.data();
    const size_t w2 = (size_t)2 * n0_;
    std::vector<int> order(n_cand);
    for (int i = 0; i < n_cand; ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](int x, int y) {
      if (parts[x] != parts[y]) return parts[x] < parts[y];
      return std::lexicographical_compare(B + x * w2, B + (x + 1) * w2, B + y * w2, B + (y + 1) * w2);
    });
    for (int i : order) {
      const int p = parts[i];
      if (!ok[i] || got[p]) continue;
      got[p] = 1;
      newly.push_back(p);
      for (int d = 0; d < n0_; ++d) {
        cex_x[(size_t)p * n0_ + d] = (int64_t)std::llround(B[(size_t)i * 2 * n0_ + d]);
        cex_xp[(size_t)p * n0_ + d] = (int64_t)std::llround(B[(size_t)i * 2 * n0_ + n0_ + d]);
      }
    }
    if (!newly.empty()) {
      idx_.ensure(newly.size());
      hidx_.ensure(newly.size() * sizeof(int));
      std::memcpy(hidx_.p, newly.data(), newly.size() * sizeof(int));
      ck(hipMemcpyAsync(idx_.p, hidx_.p, newly.size() * sizeof(int), hipMemcpyHostToDevice, st), "cp idx");
      ckl(fa_set_status_launch(idx_.p, (int)newly.size(), status_.p, 1, st), "set_status");
      // no sync: the next level's kernels are stream-ordered after set_status, and hidx_.p / idx_
      // are only rewritten by the next call, which runs after the next level-end sync (the sync
      // that retires this copy -- the buffer-lifetime rule of tests/test_stream_lifetime.py)
    }
  }

  // 1 violation, 0 not a violation, -1 undecided here (Python exact check)
  int exact_check(const float* pair, int p) const {
    return exact_.check(pair, box_lo_ + (size_t)p * n0_, box_hi_ + (size_t)p * n0_);
  }

  NetDesc net_;
  const float* flat_;
  fa_exact::ExactChecker exact_;   // fp64 host copy of the network + query constraints
  bool native_exact_ = false;
  const float* box_lo_ = nullptr;
  const float* box_hi_ = nullptr;
  std::vector<int> pa_, ra_;
  float tau_;
  int cap_, batch_, cand_cap_;
  int cand_alloc_ = 0;
  int pool_[2] = {0, 0};
  double unit_;
  bool crown_ = false;
  int refine_ = 0;          // 0 forward + output pass, 1 + refine between them, 2 backward only
  bool smear_ = false;      // first-layer smear split scores (CertArgs.smear)
  bool fuse_settle_ = fuse_settle();   // level end in the last split launch (BaBConfig.fuse_settle)
  int split_target_ = 256;
  int n0_ = 0, npa_ = 0, V_ = 0, Pp_ = 0, norient_ = 1;
  bool relaxed_ = false;
  DevBuf<float> vals_f_, w0t_;
  DevBuf<int64_t> vals_i_, pairs_;
  DevBuf<uint8_t> shared_;
  DevBuf<float> lo_[2], hi_[2], plo_[2], phi_[2];
  DevBuf<int> part_[2];
  DevBuf<float> Lc_[2], Uc_[2], L0_[2], Le_[2], U0_[2], Ue_[2], olb_[2], oub_[2], lay_lb_[2], lay_ub_[2];
  DevBuf<float> gmin_, tstar_, score_, cand_, scores_, pe_lb_, pe_ub_;
  DevBuf<uint8_t> open_, leaf_;
  DevBuf<int64_t> split_, cv_, co_;
  DevBuf<int> counters_, nodes_, idx_, open_left_, lvl_open_, nodes_start_, prev_start_, out_, pbudget_;
  DevBuf<int8_t> status_;
  DevBuf<uint8_t> prob_;
  DevBuf<unsigned char> stage_;
  fa_mem::HostBuf hcount_buf_{true};   // coherent: the settle kernel writes the level counters
  int* hcount_ = nullptr;
  // pinned host staging (solve start, solve end, per-level candidate records, confirmed-SAT
  // partition ids before fa_set_status), grown through the caching allocator (devmem.h).
  // Buffer-lifetime rule of this runtime (checked by tests/test_stream_lifetime.py): the host side
  // of EVERY hipMemcpyAsync is one of these runtime-owned pinned buffers, never a pageable
  // std::vector / numpy temporary, and nothing writes, releases or regrows it before the
  // hipStreamSynchronize that retires the copy (so a released block is idle when the cache hands
  // it to another runtime).  Round 1 enqueued pageable H2D copies and then rewrote the source
  // vector in place (relaxed x' boxes); with 8 host threads that raced the runtime's staging of
  // pageable copies.
  fa_mem::HostBuf hstage_, hout_, hidx_;
  // candidate records [cand_alloc_][2 n0 + 1], written by fa_split_kernel into coherent pinned host
  // memory and read by confirm_candidates after the level-end synchronisation; the next level's
  // split (launched after the confirmation returns) is the next writer
  fa_mem::HostBuf cand_host_{true};
};

void register_bab(py::module& m) {
  py::class_<BabRuntime>(m, "BabRuntime")
      .def(py::init<py::handle, uintptr_t, std::vector<int>, std::vector<float>, std::vector<int64_t>,
                    std::vector<int64_t>, std::vector<int>, float, std::vector<uint8_t>, int, int, int, double, bool,
                    int, int, bool>(),
           py::arg("net"), py::arg("flat"), py::arg("pa"), py::arg("values_f"), py::arg("values_i"),
           py::arg("pairs"), py::arg("ra"), py::arg("tau"), py::arg("shared"), py::arg("capacity"),
           py::arg("batch_nodes"), py::arg("cand_cap"), py::arg("unit"), py::arg("crown") = true,
           py::arg("split_target") = 256, py::arg("refine") = 0, py::arg("smear") = false)
      .def("set_fuse_settle", &BabRuntime::set_fuse_settle, py::arg("on"))
      .def("solve", &BabRuntime::solve, py::arg("lo"), py::arg("hi"), py::arg("status"), py::arg("budget"),
           py::arg("time_budget"), py::arg("dead_part"), py::arg("confirm"), py::arg("stream"),
           py::arg("native_exact") = false, py::arg("budget2") = 0, py::arg("max_w") = 0,
           py::arg("esc_steps") = std::vector<std::pair<int, int>>{});
}
