"""ReLU-phase branch-and-bound on the residue of the input-split search (stage ``relu``).

The input-split BaB (engine/bab.py) closes a node when its bounds certify it; on the narrow,
deep zero-bias networks (AC-8 13-5-5-1, AC-12 5x9 of the random-init bench) a third of the
partitions never close that way: the logit is EXACTLY 0 on a large region (every path to it
dead) and the violation needs ``N(x) < 0 < N(x')`` strictly, so any relaxation slack at the
boundary of that region -- a hypersurface through the box -- keeps nodes open however far the box
is split.  The reference decides these with Z3, whose exact simplex case-splits the ReLU
``If``s (utils/verif_utils.py:525-528, src/AC/Verify-AC.py:146-158).  This stage does the GPU
analogue:

* a node is (partition, ordered PA pair (v, v'), input box, ReLU phase of each neuron of the two
  network copies N(., v) and N(., v')); one tree per ordered pair (splits made for one pair do not
  multiply another's tree);
* bounds: forward symbolic bounds with the phases fixed (ops/reference.py:bounds ``phase``: a
  neuron fixed inactive outputs 0, one fixed active has the identity as its upper relaxation), then
  backward bounds concretised at EVERY layer with exact zeros kept (ops/reference.py:crown_phase);
* the node closes when copy v is provably >= 0 or copy v' provably <= 0 on the branch region
  (rigorous, exact zeros count), when a fixed phase contradicts the bounds (empty region), or by
  the coupled pair certificate ``min_t max_x t(-L_v(x)) + (1-t) U_v'(x) <= 0`` over the shared
  input box;
* branching: the bound (lower of N_v or upper of N_v') closest to closing, split at the unstable
  neuron whose chord intercept it pays most (BaBSR-like); when no unstable neuron is left, an
  input split (box halves) -- single lattice points are decided exactly, so the search is complete;
* every node's LP-optimal vertex pair is evaluated rigorously and confirmed exactly on the host
  (engine/exact.py): SAT answers are real counterexamples of the original network.

Every UNSAT is a proof from rigorous fp32 bounds (Higham gamma terms, outward rounding): this is
the sound replacement of the floating-point HiGHS MILP UNSAT (smt/milp.py) for these networks.
CPU measurement on the dumped residue (tools/exp/relu_proto.py): AC-8 38/40 closed with 6
nodes, AC-12 40/40 with a median of 34 nodes; AC-7 needs more (wide layers, no exact zeros).

The torch path here is the reference semantics (CPU tests); on the GPU the native runtime
(csrc/relu_runtime.cpp + csrc/relu.hip) runs the same algorithm.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from ..models.mlp import MLP
from ..ops import reference as ref
from ..ops.backend import Backend
from ..spec import ResolvedQuery
from ..utils.timer import NULL, StageTimer
from . import exact
from .bab import RUNNING, SAT, UNKNOWN, UNSAT, BaBResult, _pa_table, pa_groups


@dataclass
class ReluConfig:
    node_budget: int = 2048          # nodes per partition (all its pair trees together)
    batch_nodes: int = 32768         # nodes bounded per sub-batch (torch path: per level)
    time_budget: float = 1e9         # wall-clock seconds for the whole call
    max_pool: int = 1 << 22          # live nodes (more: the partitions losing nodes end UNKNOWN)
    # native runtime: hidden-layer bounds of every node tightened by back-substitution with its
    # fixed phases (csrc/refine.hip; a refined bound contradicting a fixed phase proves the node's
    # region empty); "auto" = BaBConfig.refine's rule.  Default off: on the bench (AC-11 is the
    # only refine-eligible net the stage runs on) it decided 3 partitions per step fewer at +3-8 %
    # step time, and on the trained AC-7 residue it closed none either way
    # (profiles/r4/relu_refine.md)
    refine: str = os.environ.get("FAIRIFY_RELU_REFINE", "off")
    # relaxed queries on the native runtime: both orientations as roots of ONE search (the reverse
    # orientation's nodes read the negated logit's forms, csrc/relu.hip) with the two solves' budgets
    # pooled, instead of a second search on the negated network for the partitions the first closed
    merge_orient: bool = os.environ.get("FAIRIFY_RELU_MERGE", "1") != "0"


def supported(q: ResolvedQuery) -> bool:
    """PA-only and relaxed queries (|x_r - x'_r| <= tau on the RA dims, x' unclipped: the nodes then
    carry a second box for the x' RA coordinates, and the second orientation runs on the negated
    network; see :meth:`ReluBaBSolver.solve`)."""
    return True


def negated(mlp: MLP) -> MLP:
    """The network with its logit negated (last layer's weights and bias): N_A > 0 > N_B on ``mlp``
    is N_A < 0 < N_B on the result -- the second orientation of a relaxed query, where x' may leave
    the box so swapping the pair does not cover it."""
    ws = [w.copy() for w in mlp.weights]
    bs = [b.copy() for b in mlp.biases]
    ws[-1] = -ws[-1]
    bs[-1] = -bs[-1]
    return MLP(ws, bs, name=mlp.name + "-neg")


def certify_pair(LA_c, LA_0, MA, UB_c, UB_0, MB, lo, hi, free, unit):
    """Coupled pair certificate of nodes with one ordered pair each.

    Violation needs L_A(x) - eL <= N_A(x) < 0 and 0 < N_B(x) <= U_B(x) + eU on the shared box;
    the node is clean if some t in [0, 1] gives  max_x t (-L_A(x)) + (1 - t) U_B(x) <= 0  (forms
    given with their errors folded into the constants: LA_0 = L0 - eL, UB_0 = U0 + eU; MA / MB =
    magnitudes for the rounding margin).  Returns (g* [N], t* [N], vertex x* [N, n0])."""
    N, n0 = lo.shape
    dt = lo.dtype
    A = -LA_c * free
    A0 = -LA_0
    B = UB_c * free
    B0 = UB_0
    den = A - B
    tb = torch.where(den.abs() > 0, -B / torch.where(den.abs() > 0, den, torch.ones_like(den)),
                     torch.full_like(den, -1.0)).clamp(-1.0, 2.0)
    ts = torch.cat([torch.zeros(N, 1, dtype=dt, device=lo.device), torch.ones(N, 1, dtype=dt, device=lo.device),
                    tb], dim=1).clamp(0.0, 1.0)                                   # [N, T]
    t = ts[:, :, None]
    cs = t * A[:, None, :] + (1 - t) * B[:, None, :]                             # [N, T, n0]
    val = torch.maximum(cs * lo[:, None, :], cs * hi[:, None, :]).sum(-1)
    g = val + ts * A0[:, None] + (1 - ts) * B0[:, None]
    g = g + ref.gamma(2 * n0 + 4, unit) * (ts * MA[:, None] + (1 - ts) * MB[:, None]) + 8 * unit * (MA + MB)[:, None]
    gmin, targ = g.min(dim=1)
    tstar = ts.gather(1, targ[:, None])[:, 0]
    c = tstar[:, None] * A + (1 - tstar[:, None]) * B
    xstar = torch.where(c > 0, hi, lo)
    return gmin, tstar, xstar


def certify_pair_relaxed(LA_c, LA_0, MA, UB_c, UB_0, MB, lo, hi, plo, phi, shared, ra, unit):
    """:func:`certify_pair` for relaxed queries: copy A reads x, copy B reads x with the RA dims
    replaced by x' (their own box [plo, phi]).  Shared dims (``shared``: non-PA, non-RA) couple the
    copies as before; on an RA dim the two maxima are taken separately (x_r in [lo, hi], x'_r in
    [plo, phi]) -- the tie |x_r - x'_r| <= tau is dropped, which only loosens the bound.  Returns
    (g*, t*, x*, x'* on the RA dims)."""
    N, n0 = lo.shape
    dt = lo.dtype
    A = -LA_c
    B = UB_c
    As, Bs = A * shared, B * shared
    den = As - Bs
    tb = torch.where(den.abs() > 0, -Bs / torch.where(den.abs() > 0, den, torch.ones_like(den)),
                     torch.full_like(den, -1.0)).clamp(-1.0, 2.0)
    ts = torch.cat([torch.zeros(N, 1, dtype=dt, device=lo.device), torch.ones(N, 1, dtype=dt, device=lo.device),
                    tb], dim=1).clamp(0.0, 1.0)                                   # [N, T]
    t = ts[:, :, None]
    cs = t * As[:, None, :] + (1 - t) * Bs[:, None, :]
    val = torch.maximum(cs * lo[:, None, :], cs * hi[:, None, :]).sum(-1)
    ar = A[:, ra][:, None, :] * t                                                 # [N, T, nra]
    br = B[:, ra][:, None, :] * (1 - t)
    val = val + torch.maximum(ar * lo[:, None, ra], ar * hi[:, None, ra]).sum(-1) \
        + torch.maximum(br * plo[:, None, :], br * phi[:, None, :]).sum(-1)
    g = val + ts * LA_0[:, None].neg() + (1 - ts) * UB_0[:, None]
    g = g + ref.gamma(2 * n0 + 4, unit) * (ts * MA[:, None] + (1 - ts) * MB[:, None]) + 8 * unit * (MA + MB)[:, None]
    gmin, targ = g.min(dim=1)
    tstar = ts.gather(1, targ[:, None])[:, 0]
    c = tstar[:, None] * A + (1 - tstar[:, None]) * B
    xstar = torch.where(c > 0, hi, lo)
    xstar[:, ra] = torch.where(A[:, ra] > 0, hi[:, ra], lo[:, ra])
    xpstar = torch.where(B[:, ra] > 0, phi, plo)
    return gmin, tstar, xstar, xpstar


def _pick_form(res_c, res_0, res_e, fw_low, cr):
    """Per row, the tighter of the forward form (res_c, res_0, res_e; its bound fw_low) and the
    backward input form ``cr`` = (coef, const, err, low)."""
    lam, c, err, low = cr
    use = (low >= fw_low)[:, None]
    return (torch.where(use, lam, res_c), torch.where(use[:, 0], c, res_0), torch.where(use[:, 0], err, res_e))


class ReluBaBSolver:
    def __init__(self, backend: Backend, query: ResolvedQuery, cfg: ReluConfig, timer: StageTimer = NULL):
        self.be = backend
        self.q = query
        self.cfg = cfg
        self.tm = timer
        self.dev = backend.device
        self.stats = {}

    def solve(self, lo_np: np.ndarray, hi_np: np.ndarray, mlp_exact: MLP,
              init_status: Optional[np.ndarray] = None) -> BaBResult:
        """Relaxed queries: orientation N(x, v) < 0 < N(x', v') on this backend's network, then, on the
        partitions it closed, N(x, v) > 0 > N(x', v') as the first orientation of the NEGATED network
        (:func:`negated`); a partition is UNSAT when both close, SAT when either finds a pair (always
        confirmed exactly on ``mlp_exact``, whose violation test is orientation-free)."""
        t0 = time.time()
        P, n = lo_np.shape
        status = np.full(P, RUNNING, dtype=np.int8) if init_status is None else init_status.astype(np.int8).copy()
        if not supported(self.q):
            status[status == RUNNING] = UNKNOWN
            return BaBResult(status, np.zeros((P, n), np.int64), np.zeros((P, n), np.int64), np.zeros(P, np.int64))
        if self.q.relaxed and not getattr(self, "_second", False) and not self._merged():
            r1 = self._solve_groups_all(lo_np, hi_np, mlp_exact, status, t0)
            closed = (r1.status == UNSAT) & (status == RUNNING)
            if not closed.any():
                return r1
            neg = ReluBaBSolver(Backend(negated(self.be.mlp), device=self.dev), self.q,
                                ReluConfig(node_budget=self.cfg.node_budget, batch_nodes=self.cfg.batch_nodes,
                                           time_budget=max(0.0, self.cfg.time_budget - (time.time() - t0)),
                                           max_pool=self.cfg.max_pool), timer=self.tm)
            neg._second = True
            st2 = np.where(closed, RUNNING, UNKNOWN).astype(np.int8)
            r2 = neg.solve(lo_np, hi_np, mlp_exact, init_status=st2)
            out = r1.status.copy()
            out[closed] = r2.status[closed]                 # UNSAT only if the second closed too
            cx, cxp = r1.cex_x.copy(), r1.cex_xp.copy()
            s2 = closed & (r2.status == SAT)
            cx[s2], cxp[s2] = r2.cex_x[s2], r2.cex_xp[s2]
            return BaBResult(out, cx, cxp, r1.nodes + r2.nodes, 0, time.time() - t0)
        return self._solve_groups_all(lo_np, hi_np, mlp_exact, status, t0)

    def _native(self) -> bool:
        torch_rx = self.q.relaxed and os.environ.get("FAIRIFY_RELU_RELAXED_TORCH") == "1"
        return self.be.hip and os.environ.get("FAIRIFY_TORCH_BAB") != "1" and not torch_rx

    def _merged(self) -> bool:
        """Relaxed query, both orientations in the native runtime's one search."""
        return self.q.relaxed and self.cfg.merge_orient and self._native()

    def _solve_groups_all(self, lo_np, hi_np, mlp_exact, status, t0) -> BaBResult:
        P, n = lo_np.shape
        status = status.copy()
        groups = pa_groups(self.q, lo_np, hi_np)
        cex_x = np.zeros((P, n), dtype=np.int64)
        cex_xp = np.zeros((P, n), dtype=np.int64)
        nodes = np.zeros(P, dtype=np.int64)
        for g in groups:
            left = max(0.0, self.cfg.time_budget - (time.time() - t0))
            st, cx, cxp, nd = self._solve_group(lo_np[g], hi_np[g], mlp_exact, status[g], left)
            status[g], cex_x[g], cex_xp[g], nodes[g] = st, cx, cxp, nd
        return BaBResult(status, cex_x, cex_xp, nodes, 0, time.time() - t0)

    # ------------------------------------------------------------------------------------------
    def _solve_group(self, lo_np, hi_np, mlp_exact, status, time_budget):
        values_np, pairs_np = _pa_table(self.q, lo_np, hi_np)
        # the native runtime (csrc/relu_runtime.cpp) on the GPU, PA-only and relaxed queries alike
        # (relaxed: an x' RA box per node; the second orientation is solve()'s negated network);
        # FAIRIFY_TORCH_BAB=1: the torch orchestration (the reference semantics of the CPU tests)
        # (FAIRIFY_RELU_RELAXED_TORCH=1: relaxed queries only, the A/B of the native relaxed path)
        if self._native():
            return self._solve_native(lo_np, hi_np, mlp_exact, status, values_np, pairs_np, time_budget)
        return self._solve_torch(lo_np, hi_np, mlp_exact, status, values_np, pairs_np, time_budget)

    def _solve_torch(self, lo_np, hi_np, mlp_exact, status, values_np, pairs_np, time_budget):
        t0 = time.time()
        be, q, cfg = self.be, self.q, self.cfg
        dev, dt = self.dev, self.be.dtype
        P, n0 = lo_np.shape
        Nh = be.n_hidden
        pa = list(q.pa_idx)
        status = status.copy()
        cex_x = np.zeros((P, n0), dtype=np.int64)
        cex_xp = np.zeros((P, n0), dtype=np.int64)
        nodes_np = np.zeros(P, dtype=np.int64)
        Pp = pairs_np.shape[0]
        run = np.nonzero(status == RUNNING)[0]
        if Pp == 0:
            status[run] = UNSAT
            return status, cex_x, cex_xp, nodes_np
        values = torch.from_numpy(values_np).to(dev, dt)
        pairs = torch.from_numpy(pairs_np).to(dev)
        free = torch.ones(n0, dtype=dt, device=dev)
        free[pa] = 0
        relaxed = q.relaxed
        ra = list(q.ra_idx) if relaxed else []
        tau = float(q.tau)
        shared = free.clone()
        shared[ra] = 0
        # one root per (partition, ordered pair)
        part = torch.from_numpy(np.repeat(run, Pp)).to(dev)
        pair = torch.arange(Pp, device=dev).repeat(len(run))
        lo = torch.from_numpy(lo_np).to(dev, dt)[part]
        hi = torch.from_numpy(hi_np).to(dev, dt)[part]
        # relaxed: the x' coordinates of the RA dims, unclipped, [lo - tau, hi + tau]
        plo = (lo[:, ra] - tau) if relaxed else torch.zeros(len(part), 0, dtype=dt, device=dev)
        phi = (hi[:, ra] + tau) if relaxed else torch.zeros(len(part), 0, dtype=dt, device=dev)
        phase = torch.zeros(len(part), 2, Nh, dtype=torch.int8, device=dev)
        levels = 0
        timed_out = False
        while part.numel():
            if time.time() - t0 > time_budget:
                timed_out = True
                break
            levels += 1
            N = part.numel()
            alive = torch.from_numpy(status == RUNNING).to(dev)[part]
            if relaxed:      # x_r and x'_r boxes more than tau apart: no admissible pair, node closed
                alive &= ~((plo > hi[:, ra] + tau) | (phi < lo[:, ra] - tau)).any(dim=1)
            if not bool(alive.all()):
                part, pair, lo, hi, phase = part[alive], pair[alive], lo[alive], hi[alive], phase[alive]
                plo, phi = plo[alive], phi[alive]
                N = part.numel()
                if N == 0:
                    break
            np.add.at(nodes_np, part.cpu().numpy(), 1)
            vA, vB = pairs[pair, 0], pairs[pair, 1]
            rlo = lo.repeat_interleave(2, dim=0)
            rhi = hi.repeat_interleave(2, dim=0)
            rv = torch.stack([vA, vB], dim=1).reshape(-1)
            rlo[:, pa] = values[rv]
            rhi[:, pa] = values[rv]
            if relaxed:          # copy B reads x' on the RA dims
                rlo[1::2, ra] = plo
                rhi[1::2, ra] = phi
            rph = phase.reshape(2 * N, Nh)
            with self.tm("relu.bounds"):
                res = be.bounds(rlo, rhi, mode="symbolic", keep_layers=True, phase=rph)
                pc, forms = be.crown_phase(rlo, rhi, res, rph)
            A, B = slice(0, None, 2), slice(1, None, 2)
            if forms is None:
                # HIP kernel: logit bounds intersected, infeasible rows set to (+inf, -inf) and the
                # tighter input forms written into ``res`` in place
                olb, oub = res.out_lb.to(dt), res.out_ub.to(dt)
                LAc, LA0, LAe = res.Lc, res.L0, res.Le
                UBc, UB0, UBe = res.Uc, res.U0, res.Ue
            else:
                olb = torch.maximum(res.out_lb.to(dt), pc.low[:, 0].to(dt))
                oub = torch.minimum(res.out_ub.to(dt), -pc.low[:, 1].to(dt))
                inf = res.infeasible if res.infeasible is not None else torch.zeros(2 * N, dtype=torch.bool,
                                                                                    device=dev)
                olb = torch.where(inf, torch.full_like(olb, float("inf")), olb)
                oub = torch.where(inf, torch.full_like(oub, -float("inf")), oub)
                # coupled certificate on the input forms (the tighter of forward / backward per row)
                LAc, LA0, LAe = _pick_form(res.Lc, res.L0, res.Le, res.out_lb, forms[1.0])
                lamU, cU, eU, lowU = forms[-1.0]
                UBc, UB0, UBe = _pick_form(res.Uc, res.U0, res.Ue, -res.out_ub, (-lamU, -cU, eU, lowU))
            closed = (olb[A] >= 0) | (oub[B] <= 0)
            LAc, LA0, LAe = LAc[A], LA0[A], LAe[A]
            UBc, UB0, UBe = UBc[B], UB0[B], UBe[B]
            # fold the PA coordinates (fixed per row) into the constants
            fa_A = (LAc[:, pa] * values[vA]).sum(1)
            fa_B = (UBc[:, pa] * values[vB]).sum(1)
            mxb = torch.maximum(lo.abs(), hi.abs())
            mxb_b = mxb.clone()
            if relaxed:
                mxb_b[:, ra] = torch.maximum(plo.abs(), phi.abs())
            # rounding margin over the folded PA products' magnitudes (with several PA dims their
            # sum can cancel below the products' errors)
            MA = (LAc.abs() * mxb * free).sum(1) + (LA0 - LAe).abs() + (LAc[:, pa] * values[vA]).abs().sum(1)
            MB = (UBc.abs() * mxb_b * free).sum(1) + (UB0 + UBe).abs() + (UBc[:, pa] * values[vB]).abs().sum(1)
            xpstar = None
            if relaxed:
                LAcf, UBcf = LAc * free, UBc * free
                g, tstar, xstar, xpstar = certify_pair_relaxed(LAcf, LA0 - LAe + fa_A, MA, UBcf, UB0 + UBe + fa_B, MB,
                                                               lo, hi, plo, phi, shared, ra, be.unit)
            else:
                g, tstar, xstar = certify_pair(LAc, LA0 - LAe + fa_A, MA, UBc, UB0 + UBe + fa_B, MB, lo, hi, free,
                                               be.unit)
            open_ = ~closed & (g > 0)
            # ---- candidate vertex pairs of open nodes: rigorous point bounds, then the exact check
            oi = torch.nonzero(open_).flatten()
            if oi.numel():
                xa = xstar[oi].clone()
                xb = xstar[oi].clone()
                xa[:, pa] = values[vA[oi]]
                xb[:, pa] = values[vB[oi]]
                if relaxed:      # x'_r: its vertex, pulled into [x_r - tau, x_r + tau]
                    xb[:, ra] = torch.minimum(torch.maximum(xpstar[oi], xa[:, ra] - tau), xa[:, ra] + tau)
                with self.tm("relu.cand"):
                    alb, _ = be.point_bounds(xa)
                    _, bub = be.point_bounds(xb)
                poss = (alb < 0) & (bub > 0)
                ci = oi[poss]
                if ci.numel():
                    self._confirm(ci, xa[poss], xb[poss], part, status, cex_x, cex_xp, mlp_exact, lo_np, hi_np)
            # ---- leaves: the non-PA box (and the x' RA box) is a single lattice point -> decided
            # exactly above
            width = ((hi - lo) * free).amax(dim=1)
            if relaxed:
                width = torch.maximum(width, (phi - plo).amax(dim=1))
            leaf = open_ & (width == 0)
            run_t = torch.from_numpy(status == RUNNING).to(dev)[part]
            grow = open_ & ~leaf & run_t
            if not bool(grow.any()):
                break
            # ---- budget: a partition past its node budget with open nodes ends UNKNOWN
            over = torch.from_numpy(nodes_np >= cfg.node_budget).to(dev)[part] & grow
            if bool(over.any()):
                status[np.unique(part[over].cpu().numpy())] = UNKNOWN
                grow = grow & ~over
            gi = torch.nonzero(grow).flatten()
            # ---- branching: the bound closest to closing, at its best neuron; else an input split
            gapA = -olb[A][gi]
            gapB = oub[B][gi]
            sA = pc.split[A, 0][gi]
            sB = pc.split[B, 1][gi]
            useA = (sA >= 0) & ((gapA <= gapB) | (sB < 0))
            useB = ~useA & (sB >= 0)
            relu = useA | useB
            row = torch.where(useA, torch.zeros_like(sA), torch.ones_like(sA))
            neu = torch.where(useA, sA, sB)
            ri = gi[relu]
            cp = phase[ri].repeat(2, 1, 1)
            k = ri.numel()
            r2 = row[relu].repeat(2)
            n2 = neu[relu].repeat(2)
            cp[torch.arange(2 * k, device=dev), r2, n2] = torch.cat([torch.full((k,), -1, dtype=torch.int8, device=dev),
                                                                     torch.ones(k, dtype=torch.int8, device=dev)])
            # input split along the dim of largest |coefficient| x width of the certificate at t*
            # (relaxed: the x' RA dims compete as extra columns, scored by copy B's coefficient)
            ii = gi[~relu]
            c_t = tstar[ii, None] * (-LAc[ii]) + (1 - tstar[ii, None]) * UBc[ii]
            if relaxed:
                c_t[:, ra] = tstar[ii, None] * LAc[ii][:, ra]
            w = (hi[ii] - lo[ii]) * free
            sc = torch.where(w > 0, c_t.abs() * w + 1e-9 * w, torch.full_like(w, -1.0))
            if relaxed:
                wp = phi[ii] - plo[ii]
                cp_ = (1 - tstar[ii, None]) * UBc[ii][:, ra]
                sc = torch.cat([sc, torch.where(wp > 0, cp_.abs() * wp + 1e-9 * wp, torch.full_like(wp, -1.0))], dim=1)
            d = sc.argmax(dim=1)
            ar = torch.arange(ii.numel(), device=dev)
            lo1, hi1, lo2, hi2 = lo[ii].clone(), hi[ii].clone(), lo[ii].clone(), hi[ii].clone()
            plo1, phi1, plo2, phi2 = plo[ii].clone(), phi[ii].clone(), plo[ii].clone(), phi[ii].clone()
            onx = d < n0
            if bool(onx.any()):
                a_, d_ = ar[onx], d[onx]
                mid = torch.floor((lo[ii][a_, d_] + hi[ii][a_, d_]) / 2)
                hi1[a_, d_] = mid
                lo2[a_, d_] = mid + 1
            if relaxed and bool((~onx).any()):
                a_, d_ = ar[~onx], d[~onx] - n0
                mid = torch.floor((plo[ii][a_, d_] + phi[ii][a_, d_]) / 2)
                phi1[a_, d_] = mid
                plo2[a_, d_] = mid + 1
            part = torch.cat([part[ri], part[ri], part[ii], part[ii]])
            pair = torch.cat([pair[ri], pair[ri], pair[ii], pair[ii]])
            lo_n = torch.cat([lo[ri], lo[ri], lo1, lo2])
            hi_n = torch.cat([hi[ri], hi[ri], hi1, hi2])
            plo = torch.cat([plo[ri], plo[ri], plo1, plo2])
            phi = torch.cat([phi[ri], phi[ri], phi1, phi2])
            phase = torch.cat([cp, phase[ii], phase[ii]])
            lo, hi = lo_n, hi_n
            if part.numel() > cfg.max_pool:
                lost = torch.unique(part[cfg.max_pool:]).cpu().numpy()
                status[lost[status[lost] == RUNNING]] = UNKNOWN
                part, pair, lo, hi, phase, plo, phi = (t[:cfg.max_pool] for t in (part, pair, lo, hi, phase, plo, phi))
        left = set(part.cpu().numpy().tolist()) if (timed_out and part.numel()) else set()
        for p in np.nonzero(status == RUNNING)[0]:
            status[p] = UNKNOWN if p in left else UNSAT
        self.stats = {"levels": levels}
        return status, cex_x, cex_xp, nodes_np

    def _confirm(self, ci, xa, xb, part, status, cex_x, cex_xp, mlp_exact, lo_np, hi_np):
        X = xa.cpu().numpy().round().astype(np.int64)
        XP = xb.cpu().numpy().round().astype(np.int64)
        parts = part[ci].cpu().numpy()
        ok = exact.check_pair_constraints(X, XP, lo_np[parts], hi_np[parts], self.q.pa_idx, self.q.ra_idx, self.q.tau)
        viol = exact.is_violation(mlp_exact, X, XP) & ok
        # each partition's witness: the first confirmed pair in (partition, lexicographic) order
        order = np.lexsort(tuple(np.concatenate([X, XP], axis=1).T[::-1]) + (parts,))
        for k in order:
            p = parts[k]
            if viol[k] and status[p] != SAT:
                status[p] = SAT
                cex_x[p], cex_xp[p] = X[k], XP[k]

    # ------------------------------------------------------------------------------------------
    def _runtime(self, values_np: np.ndarray, pairs_np: np.ndarray, n_root: int):
        """Native (C++/HIP) ReLU-phase runtime checked out of the backend's pool (engine/rtpool.py)."""
        from ..ops import ext
        from ..ops.hip import _net
        from .rtpool import checkout

        from .bab import refine_level

        rf = min(1, refine_level(self.cfg.refine, self.be.widths))
        ra = list(self.q.ra_idx) if self.q.relaxed else []
        tau = float(self.q.tau) if self.q.relaxed else 0.0
        no = 2 if self._merged() else 1
        key = (tuple(self.q.pa_idx), values_np.tobytes(), pairs_np.tobytes(), int(self.cfg.batch_nodes), rf,
               tuple(ra), tau, no)

        def make(cap):
            return ext().ReluRuntime(_net(self.be), self.be.flat.data_ptr(), list(self.q.pa_idx),
                                     values_np.astype(np.float32).reshape(-1).tolist(),
                                     pairs_np.astype(np.int64).reshape(-1).tolist(), int(cap),
                                     int(self.cfg.batch_nodes), float(self.be.unit), rf, ra, tau, no)

        return checkout(self.be, "_relu_rt", key, max(self.cfg.max_pool, 2 * n_root), make)

    def _solve_native(self, lo_np, hi_np, mlp_exact, status, values_np, pairs_np, time_budget):
        P, n0 = lo_np.shape
        from ..ops import ext
        from ..ops.hip import _net

        if not ext().relu_fits(_net(self.be)):
            # the phase kernel cannot hold this network (a layer > 256 wide or > 160 KB of LDS):
            # the stage is skipped, its partitions stay UNKNOWN for the later stages
            status = status.copy()
            status[status == RUNNING] = UNKNOWN
            return status, np.zeros((P, n0), np.int64), np.zeros((P, n0), np.int64), np.zeros(P, np.int64)
        no = 2 if self._merged() else 1
        n_root = int((status == RUNNING).sum()) * max(1, pairs_np.shape[0]) * no
        if pairs_np.shape[0] == 0:
            status = status.copy()
            status[status == RUNNING] = UNSAT
            return status, np.zeros((P, n0), np.int64), np.zeros((P, n0), np.int64), np.zeros(P, np.int64)
        q = self.q

        def confirm(parts: np.ndarray, buf: np.ndarray) -> np.ndarray:
            X = np.rint(buf[:, :n0]).astype(np.int64)
            XP = np.rint(buf[:, n0:]).astype(np.int64)
            ok = exact.check_pair_constraints(X, XP, lo_np[parts], hi_np[parts], q.pa_idx, q.ra_idx, q.tau)
            out = np.zeros(len(parts), dtype=bool)
            idx = np.nonzero(ok)[0]
            if idx.size:
                out[idx] = exact.is_violation(mlp_exact, X[idx], XP[idx])
            return out

        stream = torch.cuda.current_stream(self.dev).cuda_stream
        with self.tm("relu.native"), self._runtime(values_np, pairs_np, n_root) as rt:
            st, cx, cxp, nodes, stats = rt.solve(lo_np.astype(np.float32), hi_np.astype(np.float32), status,
                                                 int(self.cfg.node_budget) * no, float(time_budget), confirm, stream)
        self.stats = dict(stats)
        return (np.asarray(st, dtype=np.int8), np.asarray(cx), np.asarray(cxp), np.asarray(nodes, dtype=np.int64))
