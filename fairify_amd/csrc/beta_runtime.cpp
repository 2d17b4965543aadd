// Native beta-CROWN phase-split branch-and-bound driver (stage "beta"; engine/beta_bab.py is the
// torch reference semantics, csrc/beta.hip bounds a node, csrc/beta_bab.hip keeps the pool).
//
// The reference decides each partition with one Z3 query whose simplex case-splits the ReLUs
// (src/AC/Verify-AC.py:109-158, utils/verif_utils.py:525-528).  Here a partition's query is a set of
// trees -- one per (ordered PA pair, orientation) -- of nodes (box, x' box on the RA dims, phases of
// both network copies, Lagrangian parameters) in a device-resident, double-buffered node pool.  Per
// BFS level: count the level's nodes per partition (budgets), then per sub-batch of nodes: tighten the
// children's hidden-layer bounds over their box and phase region (symbolic + refine kernels with
// phases), optimise and rigorously bound every node (fa_beta_kernel), screen the concretising vertex
// pairs with rigorous point bounds, write candidates and children; then settle (trees closed, probe,
// partitions past their budget) and ONE host synchronisation; candidate pairs are confirmed exactly on
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
extern "C" int fa_refine_launch(const NetDesc& net, BoundArgs a, hipStream_t stream);
extern "C" int fa_beta_launch(const NetDesc& nd, BetaArgs a, hipStream_t stream);
extern "C" int fa_bb_count_launch(BetaPoolArgs a, hipStream_t s);
extern "C" int fa_bb_rows_launch(BetaPoolArgs a, hipStream_t s);
extern "C" int fa_bb_intersect_launch(BetaPoolArgs a, hipStream_t s);
extern "C" int fa_bb_cand_launch(BetaPoolArgs a, hipStream_t s);
extern "C" int fa_bb_split_launch(BetaPoolArgs a, hipStream_t s);
extern "C" int fa_bb_settle_launch(int R0, const int* tree_cnt, uint8_t* tree_done, const int* tree_part,
                                   int* part_closed, int P, int8_t* status, const int* part_nodes, int probe_at,
                                   uint8_t* probed, int* probe_stops, const int* counters, int* host_counts,
                                   hipStream_t s);

const NetDesc& fa_net_desc(py::handle net);

namespace {

void bck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
void bckl(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string(what) + " launch failed, code " + std::to_string(rc));
}

template <typename T>
using BBuf = fa_mem::DevBuf<T>;

// one side of the double-buffered node pool (structure of arrays)
struct Pool {
  BBuf<int> part, tree;
  BBuf<int8_t> osg, ph;
  BBuf<float> lo, hi, plo, phi, va, vb, LBA, UBA, LBB, UBB, par, t, gt;
  int cap = 0;
};

}  // namespace

class BetaRuntime {
 public:
  BetaRuntime(py::handle net, uintptr_t flat, uintptr_t wt, std::vector<int> pa, std::vector<int> ra, double tau,
              int capacity, int batch_nodes)
      : net_(fa_net_desc(net)), flat_((const float*)flat), wt_((const float*)wt), pa_(std::move(pa)),
        ra_(std::move(ra)), tau_((float)tau), cap_(capacity), batch_(batch_nodes) {
    n0_ = net_.dims[0];
    nh_ = net_.n_hidden;
    nn_ = net_.n_neurons;
    npa_ = (int)pa_.size();
    if (npa_ == 0 || npa_ > FA_MAX_PA) throw std::invalid_argument("beta runtime: bad PA");
    for (size_t q = 1; q < pa_.size(); ++q)
      if (pa_[q] <= pa_[q - 1]) throw std::invalid_argument("beta runtime: PA dims must be increasing");
    relaxed_ = !ra_.empty() && tau_ > 0.f;
    if (!relaxed_) ra_.clear();
    if ((int)ra_.size() > FA_MAX_RA) throw std::invalid_argument("beta runtime: bad RA");
    for (int d : ra_) {
      if (d < 0 || d >= n0_ || d >= 64) throw std::invalid_argument("beta runtime: RA dim out of range");
      for (int k : pa_)
        if (k == d) throw std::invalid_argument("beta runtime: RA dim is a PA dim");
    }
    if (batch_ <= 0) throw std::invalid_argument("beta runtime: batch_nodes must be > 0");
    const size_t B = (size_t)batch_;
    skip_.ensure(B); scratch_.ensure(B * 16 * nh_); bound_.ensure(B); split_.ensure(B);
    xstar_.ensure(B * n0_); xpstar_.ensure(B * n0_); binit_.ensure(2 * B);
    rlo_.ensure(2 * B * n0_); rhi_.ensure(2 * B * n0_); rpart_.ensure(2 * B);
    olb_.ensure(2 * B); oub_.ensure(2 * B); infeas_.ensure(2 * B);
    Lc_.ensure(2 * B * n0_); Uc_.ensure(2 * B * n0_); L0_.ensure(2 * B); Le_.ensure(2 * B); U0_.ensure(2 * B);
    Ue_.ensure(2 * B);
    lay_lb_.ensure(2 * B * nn_); lay_ub_.ensure(2 * B * nn_);
    cpts_.ensure(2 * B * n0_); pe_lb_.ensure(2 * B); pe_ub_.ensure(2 * B);
    counters_.ensure(8);
    hcount_buf_.ensure(4 * sizeof(int));
    hcount_ = reinterpret_cast<int*>(hcount_buf_.p);
    // fp64 host copy of the network for the exact confirmation
    int np_ = 0;
    for (int l = 0; l < net_.n_layers; ++l) np_ = std::max(np_, net_.b_off[l] + net_.dims[l + 1]);
    std::vector<float> hf(np_);
    bck(hipMemcpy(hf.data(), flat_, np_ * sizeof(float), hipMemcpyDeviceToHost), "cp weights");
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

  // roots: device pointers of R0 root nodes in the pool layout (part, osg, lo, hi, plo, phi, va, vb,
  // LBA, UBA, LBB, UBB, ph [2][NH], par [4][NH], t, gt [2][n0]; plo / phi / gt 0 unless relaxed);
  // tree_part [R0]: each root's partition.  Returns (status, cex_x, cex_xp, nodes, stats).
  py::tuple solve(std::vector<uintptr_t> roots, int R0,
                  py::array_t<int8_t, py::array::c_style | py::array::forcecast> status0,
                  py::array_t<int, py::array::c_style | py::array::forcecast> tree_part,
                  py::array_t<float, py::array::c_style | py::array::forcecast> box_lo,
                  py::array_t<float, py::array::c_style | py::array::forcecast> box_hi, int budget, int probe_at,
                  double time_budget, py::dict cfg, py::object confirm, uintptr_t stream_i,
                  py::array_t<int, py::array::c_style | py::array::forcecast> closed0) {
    hipStream_t st = (hipStream_t)stream_i;
    const auto t0 = std::chrono::steady_clock::now();
    const int P = (int)status0.shape(0);
    if (roots.size() != 16) throw std::invalid_argument("beta solve: 16 root arrays expected");
    if (tree_part.shape(0) != R0 || box_lo.ndim() != 2 || box_lo.shape(0) != P || box_lo.shape(1) != n0_ ||
        box_hi.shape(0) != P || box_hi.shape(1) != n0_)
      throw std::invalid_argument("beta solve: shape mismatch");
    if (R0 > cap_) throw std::invalid_argument("beta solve: more roots than pool capacity");
    for (int k = 0; k < R0; ++k)
      if (tree_part.data()[k] < 0 || tree_part.data()[k] >= P) throw std::invalid_argument("beta solve: bad tree_part");
    const int iters = cfg["iters"].cast<int>(), root_iters = cfg["root_iters"].cast<int>();
    const float lr_a = cfg["lr_a"].cast<float>(), lr_b = cfg["lr_b"].cast<float>(), lr_t = cfg["lr_t"].cast<float>();
    const float child_lr = cfg["child_lr"].cast<float>(), decay = cfg["decay"].cast<float>();
    const int lookahead = cfg["lookahead"].cast<int>(), beta_pos = cfg["beta_pos"].cast<int>();
    const int stall = cfg["stall"].cast<int>(), pgap = cfg["pgap"].cast<int>();
    const int warm_beta = cfg["warm_beta"].cast<int>(), tighten = cfg["tighten"].cast<int>();
    const int feas_iters = cfg.contains("feas_iters") ? cfg["feas_iters"].cast<int>() : 0;
    box_lo_ = box_lo.data();
    box_hi_ = box_hi.data();
    status_.ensure(P); nodes_.ensure(P); probed_.ensure(P); part_closed_.ensure(P);
    tree_cnt_.ensure(std::max(R0, 1)); tree_done_.ensure(std::max(R0, 1)); tree_part_.ensure(std::max(R0, 1));
    ensure_pool(0, std::max(R0, 1));
    // staged host block: status | tree_part | closed0 (trees closed before the search: the probe's
    // count) | root tree ids 0 .. R0 - 1
    if (closed0.ndim() != 1 || closed0.shape(0) != P) throw std::invalid_argument("beta solve: closed0 shape");
    const size_t o_tp = (size_t)((P + 3) & ~3), o_c0 = o_tp + (size_t)R0 * sizeof(int);
    const size_t o_ti = o_c0 + (size_t)P * sizeof(int);
    const size_t sb = o_ti + (size_t)R0 * sizeof(int);
    hstage_.ensure(sb);
    std::memcpy(hstage_.p, status0.data(), P);
    std::memcpy(hstage_.p + o_tp, tree_part.data(), (size_t)R0 * sizeof(int));
    std::memcpy(hstage_.p + o_c0, closed0.data(), (size_t)P * sizeof(int));
    int* tid = reinterpret_cast<int*>(hstage_.p + o_ti);
    for (int k = 0; k < R0; ++k) tid[k] = k;
    stage_.ensure(sb);
    bck(hipMemcpyAsync(stage_.p, hstage_.p, sb, hipMemcpyHostToDevice, st), "cp stage");
    bck(hipMemcpyAsync(status_.p, stage_.p, P, hipMemcpyDeviceToDevice, st), "cp status");
    bck(hipMemcpyAsync(tree_part_.p, stage_.p + ((P + 3) & ~3), (size_t)R0 * sizeof(int), hipMemcpyDeviceToDevice,
                       st), "cp tree_part");
    bck(hipMemsetAsync(nodes_.p, 0, P * sizeof(int), st), "memset nodes");
    bck(hipMemsetAsync(probed_.p, 0, P, st), "memset probed");
    bck(hipMemcpyAsync(part_closed_.p, stage_.p + o_c0, (size_t)P * sizeof(int), hipMemcpyDeviceToDevice, st),
        "cp closed0");
    bck(hipMemsetAsync(tree_done_.p, 0, std::max(R0, 1), st), "memset tree_done");
    bck(hipMemsetAsync(counters_.p, 0, 8 * sizeof(int), st), "memset counters");   // [2]: probe stops
    copy_roots(roots, R0, st);
    bck(hipMemcpyAsync(pool_[0].tree.p, stage_.p + o_ti, (size_t)R0 * sizeof(int), hipMemcpyDeviceToDevice, st),
        "root tree ids");
    std::vector<int64_t> cex_x((size_t)P * n0_, 0), cex_xp((size_t)P * n0_, 0);
    std::vector<char> got(P, 0);
    int cur = 0;
    long long n_in = R0;
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
        ensure_pool(nxt, (int)std::min<long long>(2 * n_in, cap_));
        ensure_cand(n_in);
        bck(hipMemsetAsync(counters_.p, 0, 2 * sizeof(int), st), "reset counters");
        bck(hipMemsetAsync(tree_cnt_.p, 0, std::max(R0, 1) * sizeof(int), st), "reset tree counts");
        // the level's nodes per partition first (the budget test of every sub-batch sees the whole level)
        for (long long s = 0; s < n_in; s += batch_) {
          BetaPoolArgs c = pool_args(cur, nxt, s, (int)std::min<long long>(batch_, n_in - s), P, budget, warm_beta);
          c.count = 1;
          bckl(fa_bb_count_launch(c, st), "beta count");
        }
        const bool root = levels == 0;
        const float sc = root ? 1.f : child_lr;
        for (long long s = 0; s < n_in; s += batch_) {
          const int nb = (int)std::min<long long>(batch_, n_in - s);
          BetaPoolArgs a = pool_args(cur, nxt, s, nb, P, budget, warm_beta);
          a.root = root ? 1 : 0;
          bckl(fa_bb_count_launch(a, st), "beta skip");          // a.count = 0: this slice's skip flags
          if (!root && tighten) tighten_slice(a, st);
          bound_slice(a, cur, s, nb, root ? root_iters : iters, lr_a * sc, lr_b * sc, lr_t * sc, decay, lookahead,
                      beta_pos, stall, pgap, st, root ? 0 : feas_iters, lr_a, lr_b, lr_t);
          bckl(fa_bb_cand_launch(a, st), "beta cand");
          screen_slice(nb, st);
          bckl(fa_bb_split_launch(a, st), "beta split");
        }
        bckl(fa_bb_settle_launch(R0, tree_cnt_.p, tree_done_.p, tree_part_.p, part_closed_.p, P, status_.p,
                                 nodes_.p, probe_at, probed_.p, counters_.p + 2, counters_.p, hcount_, st),
             "beta settle");
        bck(hipStreamSynchronize(st), "sync");
        total += n_in;
        ++levels;
        const int n_out = std::min((int)((volatile int*)hcount_)[0], pool_[nxt].cap);
        const int n_cand = std::min((int)((volatile int*)hcount_)[1], cand_alloc_);
        if (n_cand > 0) confirm_candidates(n_cand, confirm, got, cex_x, cex_xp, st);
        cur = nxt;
        n_in = n_out;
      }
    }
    // results
    const size_t hn_off = ((size_t)P + 15) & ~size_t(15);
    const size_t hc_off = hn_off + (size_t)P * sizeof(int) + 32;
    hout_.ensure(hc_off + (size_t)P * sizeof(int));
    bck(hipMemcpyAsync(hout_.p + hc_off, part_closed_.p, (size_t)P * sizeof(int), hipMemcpyDeviceToHost, st),
        "cp closed out");
    int dev_next = 0;     // the last level's child count as the device has it (the loop saw 0)
    bck(hipMemcpyAsync(hout_.p + hn_off + (size_t)P * sizeof(int) + 16, counters_.p, sizeof(int),
                       hipMemcpyDeviceToHost, st), "cp next count");
    bck(hipMemcpyAsync(hout_.p, status_.p, P, hipMemcpyDeviceToHost, st), "cp status out");
    bck(hipMemcpyAsync(hout_.p + hn_off, nodes_.p, P * sizeof(int), hipMemcpyDeviceToHost, st), "cp nodes out");
    bck(hipMemcpyAsync(hout_.p + hn_off + (size_t)P * sizeof(int), counters_.p + 2, 4 * sizeof(int),
                       hipMemcpyDeviceToHost, st), "cp probe stops");
    bck(hipStreamSynchronize(st), "sync");
    std::memcpy(&dev_next, hout_.p + hn_off + (size_t)P * sizeof(int) + 16, sizeof(int));
    const int* hclosed = reinterpret_cast<const int*>(hout_.p + hc_off);
    const int8_t* hs = reinterpret_cast<const int8_t*>(hout_.p);
    const int* hn = reinterpret_cast<const int*>(hout_.p + hn_off);
    int probe_stops = 0;
    std::memcpy(&probe_stops, hout_.p + hn_off + (size_t)P * sizeof(int), sizeof(int));
    int nan_nodes = 0, diag[2] = {0, 0};
    std::memcpy(&nan_nodes, hout_.p + hn_off + (size_t)(P + 1) * sizeof(int), sizeof(int));
    std::memcpy(diag, hout_.p + hn_off + (size_t)(P + 2) * sizeof(int), 2 * sizeof(int));
    std::vector<char> left(P, 0);
    if (timed_out && n_in > 0) {
      std::vector<int> lp((size_t)n_in);
      bck(hipMemcpy(lp.data(), pool_[cur].part.p, n_in * sizeof(int), hipMemcpyDeviceToHost), "cp left");
      for (int p : lp) left[p] = 1;
    }
    py::array_t<int8_t> status_out(P);
    py::array_t<int64_t> nodes_out(P);
    // UNSAT needs positive evidence: every (pair, orientation) tree of the partition closed on the device
    // (settle kernel) or before the search (closed0) -- a partition still running whose trees are not
    // all closed (a loop that ended early) is UNKNOWN, never UNSAT
    std::vector<int> trees(P, 0);
    for (int k = 0; k < R0; ++k) ++trees[tree_part.data()[k]];
    int unclosed = 0;
    int over = 0;
    for (int p = 0; p < P; ++p) {
      int8_t v = hs[p];
      if (got[p]) {
        v = 1;
      } else if (v == 3 || v == 4) {
        if (left[p]) {
          v = 0;
        } else if (hclosed[p] >= trees[p] + closed0.data()[p]) {
          v = 2;                                            // every node of every tree closed => UNSAT
        } else {
          v = 0;
          ++unclosed;
        }
      }
      if (v == 0 && status0.data()[p] == 3 && !got[p]) ++over;
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
    stats["probe_stop"] = probe_stops;
    stats["nan_nodes"] = nan_nodes;
    stats["root_skip_status"] = diag[0];
    stats["root_skip_tau"] = diag[1];
    stats["unknown"] = over;
    stats["unclosed"] = unclosed;
    stats["dev_next"] = (!timed_out && levels > 0) ? dev_next : 0;
    stats["time"] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return py::make_tuple(status_out, ax, axp, nodes_out, stats);
  }

 private:
  BetaPoolArgs pool_args(int cur, int nxt, long long s, int nb, int P, int budget, int warm_beta) {
    (void)P;
    Pool& c = pool_[cur];
    Pool& o = pool_[nxt];
    BetaPoolArgs a{};
    a.N = nb; a.n0 = n0_; a.nh = nh_; a.nn = nn_; a.npa = npa_;
    for (int k = 0; k < npa_; ++k) a.pa_idx[k] = pa_[k];
    a.nra = (int)ra_.size();
    for (int k = 0; k < a.nra; ++k) a.ra_idx[k] = ra_[k];
    a.tau = tau_;
    a.leaf = -(2 * n0_ + 1);
    a.warm_beta = warm_beta;
    const size_t sn = (size_t)s;
    a.part = c.part.p + sn; a.tree = c.tree.p + sn; a.osg = c.osg.p + sn;
    a.lo = c.lo.p + sn * n0_; a.hi = c.hi.p + sn * n0_;
    a.plo = relaxed_ ? c.plo.p + sn * n0_ : nullptr; a.phi = relaxed_ ? c.phi.p + sn * n0_ : nullptr;
    a.va = c.va.p + sn * npa_; a.vb = c.vb.p + sn * npa_;
    a.LBA = c.LBA.p + sn * nh_; a.UBA = c.UBA.p + sn * nh_; a.LBB = c.LBB.p + sn * nh_; a.UBB = c.UBB.p + sn * nh_;
    a.ph = c.ph.p + sn * 2 * nh_; a.par = c.par.p + sn * 4 * nh_; a.t = c.t.p + sn;
    a.gt = relaxed_ ? c.gt.p + sn * 2 * n0_ : nullptr;
    a.status = status_.p; a.part_nodes = nodes_.p; a.budget = budget; a.tree_cnt = tree_cnt_.p;
    a.skip = skip_.p;
    a.rlo = rlo_.p; a.rhi = rhi_.p; a.rpart = rpart_.p;
    a.lay_lb = lay_lb_.p; a.lay_ub = lay_ub_.p; a.infeas = infeas_.p;
    a.bound = bound_.p; a.split = split_.p; a.xstar = xstar_.p; a.xpstar = xpstar_.p; a.binit = binit_.p;
    a.cpts = cpts_.p; a.pe_lb = pe_lb_.p; a.pe_ub = pe_ub_.p;
    a.opart = o.part.p; a.otree = o.tree.p; a.oosg = o.osg.p;
    a.olo = o.lo.p; a.ohi = o.hi.p; a.oplo = relaxed_ ? o.plo.p : nullptr; a.ophi = relaxed_ ? o.phi.p : nullptr;
    a.ova = o.va.p; a.ovb = o.vb.p;
    a.oLBA = o.LBA.p; a.oUBA = o.UBA.p; a.oLBB = o.LBB.p; a.oUBB = o.UBB.p;
    a.oph = o.ph.p; a.opar = o.par.p; a.ot = o.t.p; a.ogt = relaxed_ ? o.gt.p : nullptr;
    a.count_out = counters_.p; a.cap = o.cap;
    a.nan_count = counters_.p + 3;
    a.diag = counters_.p + 4;
    a.cand_buf = reinterpret_cast<float*>(cand_host_.p); a.cand_count = counters_.p + 1; a.cand_cap = cand_alloc_;
    return a;
  }

  // phase-aware bounds of the slice's nodes (both copies), intersected with the inherited ones
  void tighten_slice(const BetaPoolArgs& a, hipStream_t st) {
    const int R = 2 * a.N;
    bckl(fa_bb_rows_launch(a, st), "beta rows");
    bck(hipMemsetAsync(infeas_.p, 0, R, st), "memset infeas");
    BoundArgs b{};
    b.flat = flat_; b.lo = rlo_.p; b.hi = rhi_.p; b.R = R; b.symbolic = 1;
    b.out_lb = olb_.p; b.out_ub = oub_.p;
    b.Lc = Lc_.p; b.L0 = L0_.p; b.Le = Le_.p; b.Uc = Uc_.p; b.U0 = U0_.p; b.Ue = Ue_.p;
    b.layer_lb = lay_lb_.p; b.layer_ub = lay_ub_.p;
    b.V = 0;
    b.skip_status = status_.p; b.skip_part = rpart_.p;
    b.phase_in = a.ph;             // node-major [n][2][nh] = row-major [2n + copy][nh]
    b.infeas = infeas_.p;
    bckl(fa_bounds_launch(net_, b, st), "beta tighten bounds");
    if (refine_ok_) {
      const int rc = fa_refine_launch(net_, b, st);
      if (rc == -1) refine_ok_ = false;
      else bckl(rc, "beta tighten refine");
    }
    bckl(fa_bb_intersect_launch(a, st), "beta intersect");
  }

  void bound_slice(const BetaPoolArgs& pa, int cur, long long s, int nb, int iters, float lr_a, float lr_b,
                   float lr_t, float decay, int lookahead, int beta_pos, int stall, int pgap, hipStream_t st,
                   int feas_iters, float flr_a, float flr_b, float flr_t) {
    Pool& c = pool_[cur];
    const size_t sn = (size_t)s;
    BetaArgs a;
    std::memset(&a, 0, sizeof(a));
    a.flat = flat_;
    a.wt = wt_;
    a.R = nb;
    a.npa = npa_;
    for (int q = 0; q < npa_; ++q) a.pa_idx[q] = pa_[q];
    a.lo = pa.lo; a.hi = pa.hi; a.va = pa.va; a.vb = pa.vb;
    a.LBA = pa.LBA; a.UBA = pa.UBA; a.LBB = pa.LBB; a.UBB = pa.UBB;
    a.phA = c.ph.p + sn * 2 * nh_;
    a.phB = a.phA + nh_;
    a.ph_stride = 2 * nh_;
    a.par = c.par.p + sn * 4 * nh_;
    a.t = c.t.p + sn;
    a.scratch = scratch_.p;
    a.iters = iters;
    a.lr_a = lr_a; a.lr_b = lr_b; a.lr_t = lr_t; a.decay = decay;
    a.lookahead = lookahead; a.beta_pos = beta_pos; a.stall = stall; a.pgap = pgap;
    a.bound = bound_.p; a.split = split_.p; a.xstar = xstar_.p; a.binit = binit_.p;
    a.xpstar = xpstar_.p;
    if (relaxed_) {
      for (int d : ra_) a.ramask |= 1ull << d;
      a.plo = pa.plo; a.phi = pa.phi;
      a.gtie = c.gt.p + sn * 2 * n0_;
      a.tau = tau_;
    }
    a.osg = pa.osg;
    a.skip = skip_.p;
    const int rc = fa_beta_launch(net_, a, st);
    if (rc != 0) throw std::runtime_error("fa_beta_kernel launch failed, code " + std::to_string(rc));
    if (feas_iters > 0) {
      // the infeasibility pass on the nodes left open (phase constraints' Lagrangian alone): closes the
      // empty regions the verified LP detects as infeasible; only bound_ can change
      a.feas = 1;
      a.iters = feas_iters;
      a.lr_a = flr_a; a.lr_b = flr_b; a.lr_t = flr_t;     // a fresh optimisation: the roots' step sizes
      const int rf = fa_beta_launch(net_, a, st);
      if (rf != 0) throw std::runtime_error("fa_beta_kernel (feas) launch failed, code " + std::to_string(rf));
    }
  }

  void screen_slice(int nb, hipStream_t st) {
    BoundArgs pb{};
    pb.flat = flat_; pb.lo = cpts_.p; pb.hi = cpts_.p; pb.R = 2 * nb; pb.symbolic = 0;
    pb.out_lb = pe_lb_.p; pb.out_ub = pe_ub_.p;
    const int prc = fa_point_try_launch(net_, pb, st);
    if (prc < 0) bckl(-prc, "beta points");
    if (prc == 0) bckl(fa_bounds_launch(net_, pb, st), "beta points (bounds)");
  }

  void copy_roots(const std::vector<uintptr_t>& r, int R0, hipStream_t st) {
    Pool& p = pool_[0];
    auto cp = [&](void* dst, uintptr_t src, size_t bytes, const char* what) {
      if (!src) {
        bck(hipMemsetAsync(dst, 0, bytes, st), what);
        return;
      }
      bck(hipMemcpyAsync(dst, (const void*)src, bytes, hipMemcpyDeviceToDevice, st), what);
    };
    const size_t R = (size_t)R0;
    cp(p.part.p, r[0], R * sizeof(int), "root part");
    cp(p.osg.p, r[1], R, "root osg");
    cp(p.lo.p, r[2], R * n0_ * sizeof(float), "root lo");
    cp(p.hi.p, r[3], R * n0_ * sizeof(float), "root hi");
    if (relaxed_) {
      cp(p.plo.p, r[4], R * n0_ * sizeof(float), "root plo");
      cp(p.phi.p, r[5], R * n0_ * sizeof(float), "root phi");
      cp(p.gt.p, r[15], R * 2 * n0_ * sizeof(float), "root gt");
    }
    cp(p.va.p, r[6], R * npa_ * sizeof(float), "root va");
    cp(p.vb.p, r[7], R * npa_ * sizeof(float), "root vb");
    cp(p.LBA.p, r[8], R * nh_ * sizeof(float), "root LBA");
    cp(p.UBA.p, r[9], R * nh_ * sizeof(float), "root UBA");
    cp(p.LBB.p, r[10], R * nh_ * sizeof(float), "root LBB");
    cp(p.UBB.p, r[11], R * nh_ * sizeof(float), "root UBB");
    cp(p.ph.p, r[12], R * 2 * nh_, "root ph");
    cp(p.par.p, r[13], R * 4 * nh_ * sizeof(float), "root par");
    cp(p.t.p, r[14], R * sizeof(float), "root t");
  }

  void ensure_pool(int i, int need) {
    Pool& p = pool_[i];
    const int want = std::min(std::max(need, 1), cap_);
    if (want <= p.cap) return;
    int n = std::max(p.cap, 1 << 12);
    while (n < want) n = (n > cap_ / 2) ? cap_ : n * 2;
    n = std::min(n, cap_);
    const size_t N = (size_t)n;
    p.part.ensure(N); p.tree.ensure(N); p.osg.ensure(N);
    p.lo.ensure(N * n0_); p.hi.ensure(N * n0_);
    if (relaxed_) { p.plo.ensure(N * n0_); p.phi.ensure(N * n0_); p.gt.ensure(N * 2 * n0_); }
    p.va.ensure(N * npa_); p.vb.ensure(N * npa_);
    p.LBA.ensure(N * nh_); p.UBA.ensure(N * nh_); p.LBB.ensure(N * nh_); p.UBB.ensure(N * nh_);
    p.ph.ensure(N * 2 * nh_); p.par.ensure(N * 4 * nh_); p.t.ensure(N);
    p.cap = n;
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
    const float* hc = reinterpret_cast<const float*>(cand_host_.p);   // written by the split kernel
    std::vector<float> buf((size_t)n_cand * 2 * n0_);
    std::vector<int> parts(n_cand);
    for (int i = 0; i < n_cand; ++i) {
      std::memcpy(buf.data() + (size_t)i * 2 * n0_, hc + (size_t)i * rec, sizeof(float) * 2 * n0_);
      std::memcpy(&parts[i], hc + (size_t)i * rec + 2 * n0_, sizeof(int));
    }
    std::vector<char> ok(n_cand, 0);
    std::vector<int> ask;
    for (int i = 0; i < n_cand; ++i) {
      if (got[parts[i]]) continue;
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
    // each partition's witness: the first confirmed pair in (partition, lexicographic pair) order
    std::vector<int> order(n_cand);
    for (int i = 0; i < n_cand; ++i) order[i] = i;
    const float* Bf = buf.data();
    const size_t w2 = (size_t)2 * n0_;
    std::sort(order.begin(), order.end(), [&](int x, int y) {
      if (parts[x] != parts[y]) return parts[x] < parts[y];
      return std::lexicographical_compare(Bf + x * w2, Bf + (x + 1) * w2, Bf + y * w2, Bf + (y + 1) * w2);
    });
    std::vector<int> newly;
    for (int i : order) {
      const int p = parts[i];
      if (!ok[i] || got[p]) continue;
      got[p] = 1;
      newly.push_back(p);
      for (int d = 0; d < n0_; ++d) {
        cex_x[(size_t)p * n0_ + d] = (int64_t)std::llround(Bf[(size_t)i * w2 + d]);
        cex_xp[(size_t)p * n0_ + d] = (int64_t)std::llround(Bf[(size_t)i * w2 + n0_ + d]);
      }
    }
    if (!newly.empty()) {
      // SAT partitions stop: their nodes are skipped from the next level on (count kernel)
      for (size_t k = 0; k < newly.size(); ++k)
        bck(hipMemsetAsync(status_.p + newly[k], 1, 1, st), "set sat");
      bck(hipStreamSynchronize(st), "sync");
    }
  }

  NetDesc net_;
  const float* flat_;
  const float* wt_;
  std::vector<int> pa_, ra_;
  float tau_ = 0.f;
  bool relaxed_ = false;
  int cap_, batch_;
  int n0_ = 0, nh_ = 0, nn_ = 0, npa_ = 0;
  bool refine_ok_ = true;
  Pool pool_[2];
  int cand_alloc_ = 0;
  fa_exact::ExactChecker exact_;
  const float* box_lo_ = nullptr;
  const float* box_hi_ = nullptr;
  BBuf<uint8_t> skip_, infeas_, probed_, tree_done_;
  BBuf<float> scratch_, xstar_, xpstar_, binit_, rlo_, rhi_, olb_, oub_, Lc_, Uc_, L0_, Le_, U0_, Ue_, lay_lb_,
      lay_ub_, cpts_, pe_lb_, pe_ub_;
  BBuf<double> bound_;
  BBuf<int> split_, rpart_, counters_, nodes_, part_closed_, tree_cnt_, tree_part_;
  BBuf<int8_t> status_;
  BBuf<unsigned char> stage_;
  fa_mem::HostBuf hcount_buf_{true};   // coherent: the settle kernel writes the level counters
  int* hcount_ = nullptr;
  // pinned staging (released / regrown only after the stream synchronisation that retires its copy)
  fa_mem::HostBuf hstage_, hout_;
  fa_mem::HostBuf cand_host_{true};   // candidate records (coherent pinned, written by the split kernel)
};

void register_beta(py::module& m) {
  py::class_<BetaRuntime>(m, "BetaRuntime")
      .def(py::init<py::handle, uintptr_t, uintptr_t, std::vector<int>, std::vector<int>, double, int, int>(),
           py::arg("net"), py::arg("flat"), py::arg("wt"), py::arg("pa"), py::arg("ra"), py::arg("tau"),
           py::arg("capacity"), py::arg("batch_nodes"))
      .def("solve", &BetaRuntime::solve, py::arg("roots"), py::arg("R0"), py::arg("status"), py::arg("tree_part"),
           py::arg("box_lo"), py::arg("box_hi"), py::arg("budget"), py::arg("probe_at"), py::arg("time_budget"),
           py::arg("cfg"), py::arg("confirm"), py::arg("stream"), py::arg("closed0"));
}
