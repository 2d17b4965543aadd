"""LP branch-and-bound with rigorously verified dual certificates (stage ``lp``).

The reference decides every partition with Z3 (exact rationals; utils/verif_utils.py:525-528,
src/AC/Verify-AC.py:127-163).  Round 2 used a HiGHS MILP on the residue, whose UNSAT is HiGHS's
floating-point branch-and-cut dual bound -- no proof (smt/milp.py).  This stage keeps HiGHS as an
UNTRUSTED oracle and checks what it returns:

* per ordered PA pair (v, v'): the LP relaxation of the two-copy encoding of smt/milp.py
  (maximise t s.t. t <= -N(x, v), t <= N(x', v'); x real in the partition box; each unstable
  neuron's big-M binary relaxed to [0, 1], i.e. the triangle relaxation over the GPU's rigorous
  per-layer bounds; stable neurons exact).  ``t* > 0`` is necessary for a violation.
* the LP is solved by HiGHS (SciPy's bundled bindings: one persistent model per pair, dual
  simplex warm-started from the parent node's basis -- ~1.5 ms per AC-7 node instead of ~22 ms
  for a cold ``linprog``); its row multipliers y are then used in the weak-duality bound
  t <= sum_r (y_r rhi_r if y_r > 0 else y_r rlo_r) + sum_j max(r_j l_j, r_j u_j),  r = c - A^T y,
  valid for ANY y (:func:`certified_bound_rows`).  An 'infeasible' answer is accepted only with
  a certificate as well: the elastic phase-1 LP (min total row violation) must have a certified
  optimum > 0; otherwise the node is split like any open node.  The bound is evaluated in fp64 with a
  rigorous rounding term (Higham gamma_k over every dot product and the final sum), so the
  certificate does not depend on the solver being right -- only on the constraint data, which is
  exact: float32 weights / biases / GPU bounds are exact in fp64, and every constant is carried by
  a variable fixed to 1 (no rounded right-hand sides).
* a node whose certified bound is <= 0 is closed (no x with N(x, v) < 0 < N(x', v'));
  otherwise it branches on the unstable neuron whose relaxation the LP optimum exploits most
  (largest h - relu(z) at the LP point, ties: lower index), fixing its binary to 0 / 1 -- the
  exact phase constraints -- and, with no unstable neuron left, splits the widest input dimension
  of the integer box (lattice points are decided exactly, so the search is complete);
* the LP primal point, rounded to the lattice, is a counterexample candidate: the pipeline
  confirms it with the exact checker before counting a SAT.

Cost: one small warm-started LP per node (~341 variables, 322 rows for AC-7) on the host; the stage runs in the anytime mode (Table V), where the round-2 MILP ran.  CPU tests pin
its verdicts to brute-force lattice enumeration (tests/test_lpbab.py).
"""
from __future__ import annotations

import heapq
import math
import threading
import time
from typing import List, Optional, Sequence, Tuple

import numpy as np

U64 = 2.0 ** -53


def _gamma(k: int) -> float:
    ku = k * U64
    return ku / (1.0 - ku)


class _LP:
    """Two-copy LP of one ordered PA pair with exact data.  Variables: [one | x (n0) | PA dims of
    x' | RA dims of x' (relaxed queries) | per copy and layer: h (w_l), a (unstable) | t]; rows
    two-sided (lo <= A v <= hi)."""

    def __init__(self, weights, biases, lo, hi, pa_idx, va, vb, bounds_a, bounds_b, sign: int = 0,
                 ra_idx: Sequence[int] = (), tau: float = 0.0, orient: int = 1):
        """``sign`` = 0: the pair LP (maximise t, t <= -N(x, va), t <= N(x', vb)); ``sign`` = -1 / +1:
        ONE copy, maximise t with t <= -N(x, va) / t <= N(x, va) (a certified t <= 0 proves that
        no point of the box has N(x, va) < 0 / > 0).

        Relaxed queries (``ra_idx``, ``tau`` > 0; reference semantics relaxed/BM/Verify-BM.py:53-54,
        utils/verif_utils.py:879-887): x' has its own integer variable on every RA dim, NOT clipped
        to the partition box (range [lo - tau, hi + tau]), tied to x by -tau <= x'_r - x_r <= tau;
        ``bounds_b`` are then the per-layer bounds over that widened box.  ``orient`` = -1: the
        other orientation, t <= N(x, va), t <= -N(x', vb) (with x' outside the box, swapping the
        pair does not cover it as it does for PA-only queries)."""
        self.nv = 0
        self.lb: List[float] = []
        self.ub: List[float] = []
        ri, rj, rv, rlo, rhi = [], [], [], [], []
        self.nr = 0

        def var(lb, ub):
            lb = np.atleast_1d(np.asarray(lb, np.float64))
            ub = np.atleast_1d(np.asarray(ub, np.float64))
            idx = np.arange(self.nv, self.nv + lb.size)
            self.nv += lb.size
            self.lb.extend(lb.tolist())
            self.ub.extend(ub.tolist())
            return idx

        def row(js, vs, lo_, hi_):
            ri.append(np.full(len(js), self.nr, np.int64))
            rj.append(np.asarray(js, np.int64))
            rv.append(np.asarray(vs, np.float64))
            rlo.append(lo_)
            rhi.append(hi_)
            self.nr += 1

        n0 = lo.size
        pa = list(pa_idx)
        self.one = var([1.0], [1.0])[0]
        self.one2 = var([1.0], [1.0])[0]        # second constant: -b and +lb stay separate exact terms
        xlo = lo.astype(np.float64).copy()
        xhi = hi.astype(np.float64).copy()
        xlo[pa] = va
        xhi[pa] = va
        self.x = var(xlo, xhi)
        xb = self.x.copy()
        xpa = var(np.asarray(vb, np.float64), np.asarray(vb, np.float64))
        for k, d in enumerate(pa):
            xb[d] = xpa[k]
        self.ra = [int(d) for d in ra_idx] if (tau > 0 and not sign) else []
        self.tau = float(tau)
        self.xr = np.zeros(0, np.int64)
        if self.ra:
            self.xr = var(lo[self.ra].astype(np.float64) - tau, hi[self.ra].astype(np.float64) + tau)
            for k, d in enumerate(self.ra):
                xb[d] = self.xr[k]
                row([self.xr[k], self.x[d]], [1.0, -1.0], -float(tau), float(tau))
        self.pa = pa
        self.vb = np.asarray(vb, np.int64)
        self.a_vars: List[Tuple[int, int, int, int, int]] = []   # (a var, h var, copy, layer, neuron)
        self.z_rows = []                                       # (copy, layer, neuron) -> (h, prev, W col, b)
        outs = []
        copies = ((self.x, bounds_a),) if sign else ((self.x, bounds_a), (xb, bounds_b))
        for cp, (xin, (lbs, ubs)) in enumerate(copies):
            prev = xin
            L = len(weights)
            for l in range(L - 1):
                W = np.asarray(weights[l], np.float64)
                b = np.asarray(biases[l], np.float64)
                lb = np.asarray(lbs[l], np.float64)
                ub = np.asarray(ubs[l], np.float64)
                w = W.shape[1]
                dead = ub <= 0
                h = var(np.zeros(w), np.where(dead, 0.0, np.maximum(ub, 0.0)))
                for j in range(w):
                    if dead[j]:
                        continue
                    js = np.concatenate([[h[j]], prev, [self.one]])
                    base = np.concatenate([[1.0], -W[:, j], [-b[j]]])       # h - W.prev - b
                    if lb[j] >= 0:
                        row(js, base, 0.0, 0.0)                             # h = z
                        continue
                    a = var([0.0], [1.0])[0]
                    self.a_vars.append((a, h[j], cp, l, j))
                    row(js, base, 0.0, np.inf)                              # h >= z
                    # h - z - lb a + lb <= 0   (h <= z - lb (1 - a))
                    row(np.concatenate([js, [self.one2, a]]), np.concatenate([base, [lb[j]], [-lb[j]]]),
                        -np.inf, 0.0)
                    row([h[j], a], [1.0, -ub[j]], -np.inf, 0.0)             # h <= ub a
                    self.z_rows.append((h[j], prev, W[:, j], b[j], lb[j], ub[j]))
                prev = h
            outs.append((prev, np.asarray(weights[-1], np.float64)[:, 0], float(np.asarray(biases[-1])[0])))
        # bound on |t|: valid because t <= N(x', v') <= its output bound, and any lower bound below
        # min(-N, N') keeps every feasible point (t is maximised)
        if sign:
            outs.append(outs[0])
        (pa_h, wa, ba), (pb_h, wb, bb) = outs
        M = 1.0 + abs(ba) + abs(bb) + float(np.abs(wa) @ np.maximum(np.asarray(self.ub)[pa_h], 0)) \
            + float(np.abs(wb) @ np.maximum(np.asarray(self.ub)[pb_h], 0))
        M = float(np.nextafter(2.0 * M, np.inf))
        self.t = var([-M], [M])[0]
        o = 1.0 if (sign or orient >= 0) else -1.0
        if sign <= 0:    # t <= -o N(x, va)
            row(np.concatenate([[self.t], pa_h, [self.one]]), np.concatenate([[1.0], o * wa, [o * ba]]), -np.inf, 0.0)
        if sign >= 0:    # t <= o N(x', vb)  (sign mode: N(x, va))
            row(np.concatenate([[self.t], pb_h, [self.one]]), np.concatenate([[1.0], -o * wb, [-o * bb]]), -np.inf,
                0.0)
        from scipy.sparse import coo_matrix

        self.A = coo_matrix((np.concatenate(rv), (np.concatenate(ri), np.concatenate(rj))),
                            shape=(self.nr, self.nv)).tocsr()
        self.rlo = np.asarray(rlo, np.float64)
        self.rhi = np.asarray(rhi, np.float64)
        self.lb = np.asarray(self.lb)
        self.ub = np.asarray(self.ub)
        self.n0 = n0
        self.c = np.zeros(self.nv)
        self.c[self.t] = -1.0
        self._h = None          # persistent HiGHS model (warm starts), built on the first solve
        self._h1 = None         # its elastic phase-1 twin (infeasibility certificates)
        # integer input variables: the non-PA dims of x, then the RA dims of x' -- a node whose
        # integer variables are all fixed is one lattice pair, decided exactly
        isx = np.ones(n0, bool)
        isx[pa] = False
        self.ivars = np.concatenate([self.x[isx], self.xr]).astype(np.int64)

    def pair(self, v: np.ndarray, lb: np.ndarray, ub: np.ndarray):
        """Lattice pair (x, x') from a variable vector (rounded into the node's bounds; x'_r also
        into x_r +- tau), PA dims of x' = vb."""
        xs = np.clip(np.rint(v[self.x]), lb[self.x], ub[self.x]).astype(np.int64)
        xps = xs.copy()
        xps[self.pa] = self.vb
        for k, d in enumerate(self.ra):
            j = self.xr[k]
            lo_ = max(lb[j], xs[d] - self.tau)
            hi_ = min(ub[j], xs[d] + self.tau)
            xps[d] = int(np.clip(np.rint(v[j]), lo_, max(lo_, hi_)))
        return xs, xps

    # ------------------------------------------------------------------------------------------
    def _highs(self, elastic: bool):
        """HiGHS model of this LP (``elastic``: every row r gets p_r, n_r >= 0 with
        rlo <= A_r v + p_r - n_r <= rhi, objective min sum(p + n))."""
        from scipy.optimize._highspy import _core as hc

        A = self.A
        c = self.c
        lb, ub = self.lb, self.ub
        if elastic:
            from scipy.sparse import eye, hstack

            I = eye(self.nr, format="csr")
            A = hstack([A, I, -I]).tocsr()
            c = np.concatenate([np.zeros(self.nv), np.ones(2 * self.nr)])
            lb = np.concatenate([lb, np.zeros(2 * self.nr)])
            ub = np.concatenate([ub, np.full(2 * self.nr, np.inf)])
        Ac = A.tocsc()
        inf = hc.kHighsInf
        h = hc._Highs()
        h.setOptionValue("output_flag", False)
        lp = hc.HighsLp()
        lp.num_col_ = A.shape[1]
        lp.num_row_ = A.shape[0]
        lp.col_cost_ = c
        lp.col_lower_ = np.where(np.isfinite(lb), lb, -inf)
        lp.col_upper_ = np.where(np.isfinite(ub), ub, inf)
        lp.row_lower_ = np.where(np.isfinite(self.rlo), self.rlo, -inf)
        lp.row_upper_ = np.where(np.isfinite(self.rhi), self.rhi, inf)
        lp.a_matrix_.format_ = hc.MatrixFormat.kColwise
        lp.a_matrix_.start_ = Ac.indptr
        lp.a_matrix_.index_ = Ac.indices
        lp.a_matrix_.value_ = Ac.data
        lp.a_matrix_.num_col_ = A.shape[1]
        lp.a_matrix_.num_row_ = A.shape[0]
        h.passModel(lp)
        return h, A, c, lb, ub, hc

    def solve(self, lb: np.ndarray, ub: np.ndarray, basis=None):
        """LP with variable bounds (lb, ub) (binaries fixed by the node) -> (t_lp or None,
        certified upper bound on t, primal v or None, basis for the children's warm start).

        HiGHS (dual simplex, warm-started from the parent's basis: ~1 pivot per child) is an
        untrusted oracle; the bound is :func:`certified_bound_rows` of its row multipliers.  An
        'infeasible' claim is only accepted with a certificate too: the elastic phase-1 LP
        (min total row violation) must have a certified optimum > 0 (weak duality on it proves
        that no v satisfies the rows within the node's bounds).  Anything uncertified returns an
        infinite bound (the caller keeps the node open)."""
        if self._h is None:
            self._h = self._highs(False)
        h, A, c, _, _, hc = self._h
        idx = np.arange(self.nv, dtype=np.int32)
        h.changeColsBounds(self.nv, idx, lb, ub)
        if basis is not None:
            h.setBasis(basis)
        h.run()
        st = h.getModelStatus()
        if st == hc.HighsModelStatus.kInfeasible:
            return None, (-math.inf if self._infeasible_certified(lb, ub) else math.inf), None, None
        if st != hc.HighsModelStatus.kOptimal:
            return None, math.inf, None, None
        sol = h.getSolution()
        y = np.asarray(sol.row_dual, np.float64)
        # max t = max (-c).v; the sign convention of HiGHS's row duals does not matter: any
        # multipliers give a valid bound, keep the better of the two readings
        cert = min(certified_bound_rows(-c, A, self.rlo, self.rhi, -y, lb, ub),
                   certified_bound_rows(-c, A, self.rlo, self.rhi, y, lb, ub))
        x = np.asarray(sol.col_value, np.float64)
        return float(x[self.t]), cert, x, h.getBasis()

    def _infeasible_certified(self, lb, ub) -> bool:
        if self._h1 is None:
            self._h1 = self._highs(True)
        h, A, c, lb1, ub1, hc = self._h1
        lbe = np.concatenate([lb, lb1[self.nv:]])
        ube = np.concatenate([ub, ub1[self.nv:]])
        n = lbe.size
        h.changeColsBounds(n, np.arange(n, dtype=np.int32), lbe, ube)
        h.run()
        if h.getModelStatus() != hc.HighsModelStatus.kOptimal:
            return False
        # the elastic columns cost 1, so optimal multipliers sit in [-1, 1] and rows at +-1 leave
        # reduced costs of exactly 0 on columns without an upper bound: shrink them a little so
        # that the rounding interval of those reduced costs stays below 0
        y = np.asarray(h.getSolution().row_dual, np.float64) * (1.0 - 1e-7)
        # max -(sum p + n) <= cert < 0  =>  every v violates some row
        cert = min(certified_bound_rows(-c, A, self.rlo, self.rhi, -y, lbe, ube),
                   certified_bound_rows(-c, A, self.rlo, self.rhi, y, lbe, ube))
        return cert < 0.0


def certified_bound(c, A_ub, b_ub, A_eq, b_eq, y_ub, y_eq, lb, ub) -> float:
    """Rigorous upper bound on  max c.v  s.t.  A_ub v <= b_ub, A_eq v = b_eq, lb <= v <= ub,
    from ANY multipliers y_ub >= 0, y_eq (weak duality), evaluated in fp64 with Higham gamma
    terms on every dot product and sum.  Infinite if a variable with an infinite bound keeps a
    nonzero reduced coefficient."""
    y_ub = np.maximum(np.asarray(y_ub, np.float64), 0.0)
    y_eq = np.asarray(y_eq, np.float64)
    m = A_ub.shape[0] + (A_eq.shape[0] if A_eq is not None else 0)
    ATy = A_ub.T @ y_ub if A_ub.shape[0] else np.zeros(len(c))
    ATy_abs = abs(A_ub).T @ y_ub if A_ub.shape[0] else np.zeros(len(c))
    if A_eq is not None and A_eq.shape[0]:
        ATy = ATy + A_eq.T @ y_eq
        ATy_abs = ATy_abs + abs(A_eq).T @ np.abs(y_eq)
    r = np.asarray(c, np.float64) - ATy
    g = 2.0 * _gamma(m + 2)                                  # x2: the rounding of ATy_abs itself
    er = g * (np.abs(c) + ATy_abs)                          # |r_fl - r_exact| <= er
    r_hi, r_lo = r + er, r - er                             # r_exact in [r_lo, r_hi] (up to the
    # rounding of these two additions, covered by the 2x slack below)
    lb = np.asarray(lb, np.float64)
    ub = np.asarray(ub, np.float64)
    # max over v_j in [lb_j, ub_j] and r_j in [r_lo, r_hi] of r_j v_j: the four corners
    with np.errstate(invalid="ignore", over="ignore"):
        corners = np.stack([r_lo * lb, r_lo * ub, r_hi * lb, r_hi * ub])
    corners = np.where(np.isnan(corners), 0.0, corners)      # 0 * inf: the coefficient is exactly 0
    term = corners.max(0)
    exact_zero = (r_lo == 0.0) & (r_hi == 0.0)
    term[exact_zero] = 0.0
    if not np.all(np.isfinite(term)):
        return math.inf
    parts = [y_ub * np.asarray(b_ub, np.float64), term]
    if A_eq is not None and A_eq.shape[0]:
        parts.append(y_eq * np.asarray(b_eq, np.float64))
    allp = np.concatenate(parts)
    s = float(np.sum(allp))
    k = allp.size + 4
    # rounding of the selected products: infinite corners (r < 0 times an unbounded side: -inf)
    # are never the maximum, so only the finite ones contribute magnitude
    cabs = np.where(np.isfinite(corners), np.abs(corners), 0.0).max(0)
    cabs[exact_zero] = 0.0
    slack = 2.0 * _gamma(k) * float(np.sum(np.abs(allp))) + 2.0 * _gamma(3) * float(np.sum(cabs))
    bound = s + slack
    return float(np.nextafter(bound, np.inf)) if math.isfinite(bound) else math.inf


def certified_bound_rows(d, A, rlo, rhi, lam, lb, ub) -> float:
    """Rigorous upper bound on  max d.v  s.t.  rlo <= A v <= rhi, lb <= v <= ub  from ANY row
    multipliers ``lam`` (either sign): d.v = (d - A^T lam).v + lam.(A v) <= sum_j max_v r_j v_j
    + sum_r (lam_r rhi_r if lam_r > 0 else lam_r rlo_r).  A multiplier whose side of its row is
    unbounded is dropped (set to 0).  fp64 with Higham gamma terms as in :func:`certified_bound`."""
    lam = np.asarray(lam, np.float64)
    rlo = np.asarray(rlo, np.float64)
    rhi = np.asarray(rhi, np.float64)
    lam = np.where(((lam > 0) & ~np.isfinite(rhi)) | ((lam < 0) & ~np.isfinite(rlo)) | ~np.isfinite(lam), 0.0, lam)
    m = A.shape[0]
    ATl = A.T @ lam if m else np.zeros(len(d))
    ATl_abs = abs(A).T @ np.abs(lam) if m else np.zeros(len(d))
    r = np.asarray(d, np.float64) - ATl
    g = 2.0 * _gamma(m + 2)
    er = g * (np.abs(d) + ATl_abs)
    r_hi, r_lo = r + er, r - er
    lb = np.asarray(lb, np.float64)
    ub = np.asarray(ub, np.float64)
    with np.errstate(invalid="ignore", over="ignore"):
        corners = np.stack([r_lo * lb, r_lo * ub, r_hi * lb, r_hi * ub])
    corners = np.where(np.isnan(corners), 0.0, corners)
    term = corners.max(0)
    exact_zero = (r_lo == 0.0) & (r_hi == 0.0)
    term[exact_zero] = 0.0
    if not np.all(np.isfinite(term)):
        return math.inf
    with np.errstate(invalid="ignore"):
        rowterm = np.where(lam > 0, lam * rhi, np.where(lam < 0, lam * rlo, 0.0))
    rowterm = np.where(lam == 0, 0.0, rowterm)
    allp = np.concatenate([rowterm, term])
    if not np.all(np.isfinite(allp)):
        return math.inf
    s = float(np.sum(allp))
    k = allp.size + 4
    # rounding of the selected products: infinite corners (r < 0 times an unbounded side: -inf)
    # are never the maximum, so only the finite ones contribute magnitude
    cabs = np.where(np.isfinite(corners), np.abs(corners), 0.0).max(0)
    cabs[exact_zero] = 0.0
    slack = 2.0 * _gamma(k) * float(np.sum(np.abs(allp))) + 2.0 * _gamma(3) * float(np.sum(cabs))
    bound = s + slack
    return float(np.nextafter(bound, np.inf)) if math.isfinite(bound) else math.inf


def _lp_bab(lp: "_LP", pa, va, node_budget: int, deadline: float, hit) -> Tuple[str, Optional[tuple], int]:
    """Best-first LP branch-and-bound over ``lp``: ('closed', None, nodes) when every node closed,
    ('hit', (x, x'), nodes) when ``hit(x, x')`` (integers, PA dims = va / vb) accepted a lattice
    pair (a leaf, or the rounded LP optimum of a node whose LP value is > 0), ('unknown', None,
    nodes) at the node budget / deadline."""
    iv = lp.ivars
    tried = set()

    def check(xs, xps) -> bool:
        key = xs.tobytes() + xps.tobytes()
        if key in tried:
            return False
        tried.add(key)
        return bool(hit(xs, xps))

    heap = [(0.0, 0, lp.lb.copy(), lp.ub.copy(), None)]   # best-first on the certified bound;
    # each entry carries its parent's simplex basis (a child differs by one bound: ~1 pivot)
    tick = 1
    nodes = 0
    while heap:
        if nodes >= node_budget or time.time() > deadline:
            return "unknown", None, nodes
        _, _, nlb, nub, pbasis = heapq.heappop(heap)
        nodes += 1
        if bool(np.all(nlb[iv] == nub[iv])):
            # a single lattice pair: decided exactly (the LP's rounding slack cannot close an
            # exactly-zero logit, the exact checker can); the pair constraints are the checker's
            xs, xps = lp.pair(nlb, nlb, nub)
            if check(xs, xps):
                return "hit", (xs, xps), nodes
            continue
        t_lp, cert, v, basis = lp.solve(nlb, nub, pbasis)
        if cert <= 0.0:
            continue
        if t_lp is not None and t_lp > 0:
            xs, xps = lp.pair(v, nlb, nub)
            if check(xs, xps):
                return "hit", (xs, xps), nodes
        # branch: the unfixed binary whose relaxation the LP optimum exploits most
        best, bi = 0.0, -1
        for i, (a, h, cp, l, j) in enumerate(lp.a_vars if v is not None else ()):
            if nlb[a] == nub[a]:
                continue
            hv, prev, wcol, bj, zl, zu = lp.z_rows[i]
            gap = float(v[h]) - max(float(v[prev] @ wcol + bj), 0.0)
            if gap > best + 1e-12:
                best, bi = gap, i
        children = []
        if bi >= 0 and best > 1e-9:
            a = lp.a_vars[bi][0]
            for val in (0.0, 1.0):
                clb, cub = nlb.copy(), nub.copy()
                clb[a] = cub[a] = val
                children.append((clb, cub))
        else:
            # the relaxation is not what keeps the node open (or the LP gave no certified answer:
            # an uncertified 'infeasible'): split the widest integer input variable (x, or x' on
            # a relaxed dim)
            wdt = nub[iv] - nlb[iv]
            j = int(iv[int(np.argmax(wdt))])
            mid = math.floor(0.5 * (nlb[j] + nub[j]))
            for lo_d, hi_d in ((nlb[j], mid), (mid + 1, nub[j])):
                clb, cub = nlb.copy(), nub.copy()
                clb[j], cub[j] = lo_d, hi_d
                children.append((clb, cub))
        for clb, cub in children:
            heapq.heappush(heap, (-cert, tick, clb, cub, basis))
            tick += 1
    return "closed", None, nodes


def lp_bab_pair(weights, biases, lo, hi, pa_idx, va, vb, bounds_a, bounds_b, node_budget: int, deadline: float,
                confirm, ra_idx: Sequence[int] = (), tau: float = 0.0, orient: int = 1
                ) -> Tuple[str, Optional[tuple], int]:
    """LP branch-and-bound of one ordered PA pair (v, v'): ('unsat', None, nodes) when every node
    closed, ('sat', (x, x'), nodes) with an exactly confirmed pair (``confirm(x, x') -> bool``),
    ('unknown', None, nodes) at the node budget / deadline.  Relaxed queries: ``ra_idx`` / ``tau``
    (x' free on the RA dims within tau of x, ``bounds_b`` over the widened box)."""
    lp = _LP(weights, biases, lo, hi, pa_idx, va, vb, bounds_a, bounds_b, ra_idx=ra_idx, tau=tau, orient=orient)
    st, wit, nodes = _lp_bab(lp, list(pa_idx), va, node_budget, deadline, confirm)
    if st == "hit":
        return "sat", (wit[0].tolist(), wit[1].tolist()), nodes
    return ("unsat" if st == "closed" else "unknown"), None, nodes


def lp_sign_free(weights, biases, lo, hi, pa_idx, va, bounds_a, sign: int, node_budget: int, deadline: float,
                 exact_sign) -> Tuple[bool, int]:
    """Single-copy LP branch-and-bound: True when no lattice point of the box (PA dims = va) has
    sign(N(x, va)) == ``sign`` (-1 / +1) -- certified by the same weak-duality bounds, leaves by
    ``exact_sign(x) -> -1 / 0 / +1``."""
    lp = _LP(weights, biases, lo, hi, pa_idx, va, va, bounds_a, bounds_a, sign=sign)
    st, _, nodes = _lp_bab(lp, list(pa_idx), va, node_budget, deadline, lambda xs, xps: exact_sign(xs) == sign)
    return st == "closed", nodes


def solve_partition(weights, biases, lo, hi, pa_idx, values, pairs, row_bounds, node_budget: int,
                    time_limit: float, confirm, exact_sign=None, ra_idx: Sequence[int] = (), tau: float = 0.0,
                    row_bounds_p=None) -> Tuple[str, Optional[tuple], int]:
    """Decide one partition over all ordered PA pairs: 'unsat' (every pair's LP-BaB closed),
    'sat' with an exactly confirmed pair (``confirm(x, x') -> bool``), else 'unknown'.

    With more than two ordered pairs (a PA of 3+ values: race has 5, i.e. 20 pairs) and
    ``exact_sign(x) -> -1/0/+1`` given, each value first gets two single-copy sign tests: a value
    v whose logit is certainly never < 0 on the box closes every pair (v, .), one whose logit is
    never > 0 closes every pair (., v) -- 2V half-size searches shared by V(V-1) pairs.

    Relaxed queries (``ra_idx``, ``tau`` > 0): x' ranges over the box widened by tau on the RA dims
    (``row_bounds_p``: per-layer bounds over it); the 'never > 0' test of x' runs on that box."""
    deadline = time.time() + time_limit
    nodes = 0
    relaxed = tau > 0 and len(ra_idx) > 0
    rbp = row_bounds_p if (relaxed and row_bounds_p is not None) else row_bounds
    if relaxed and row_bounds_p is None:
        raise ValueError("relaxed query: row_bounds_p (bounds over the widened x' box) required")
    lo_p, hi_p = lo.astype(np.float64).copy(), hi.astype(np.float64).copy()
    if relaxed:
        lo_p[list(ra_idx)] -= tau
        hi_p[list(ra_idx)] += tau
    # free[(box, sign)][v]: no lattice point of the box (x: "x", widened x' box: "p") has
    # sign(N(., v)) == sign
    free = {("x", -1): {}, ("x", 1): {}, ("p", -1): {}, ("p", 1): {}}
    if exact_sign is not None and len(pairs) > 2:
        vals = sorted({int(v) for pr in pairs for v in pr})
        tests = [("x", -1), ("p", 1)] + ([("x", 1), ("p", -1)] if relaxed else [])
        sb = max(16, node_budget // (4 * len(tests) * len(vals)))
        for v in vals:
            def es(xs, v=v):
                return exact_sign(xs)
            for box, sg in tests:
                bl, bh, rbv = (lo, hi, row_bounds[v]) if box == "x" else (lo_p, hi_p, rbp[v])
                free[(box, sg)][v], n1 = lp_sign_free(weights, biases, bl, bh, pa_idx, values[v], rbv, sg, sb,
                                                      deadline, es)
                nodes += n1
    # orientation +1: N(x, vi) < 0 < N(x', vj); -1 (relaxed only): N(x, vi) > 0 > N(x', vj)
    for orient in ((1, -1) if relaxed else (1,)):
        for vi, vj in pairs:
            if orient > 0 and (free[("x", -1)].get(int(vi)) or free[("p", 1)].get(int(vj))):
                continue
            if orient < 0 and (free[("x", 1)].get(int(vi)) or free[("p", -1)].get(int(vj))):
                continue
            st, wit, n = lp_bab_pair(weights, biases, lo, hi, pa_idx, values[int(vi)], values[int(vj)],
                                     row_bounds[int(vi)], rbp[int(vj)], max(1, node_budget - nodes), deadline,
                                     confirm, ra_idx=ra_idx if relaxed else (), tau=tau if relaxed else 0.0,
                                     orient=orient)
            nodes += n
            if st == "sat":
                return "sat", wit, nodes
            if st != "unsat":
                return "unknown", None, nodes
    return "unsat", None, nodes


_PPOOL = None
_PPOOL_N = 0
_PPOOL_LOCK = threading.Lock()


def process_pool(workers: int):
    """Worker processes of the LP stage (spawned children: numpy / SciPy only, no GPU context).
    HiGHS through SciPy keeps the GIL, so threads do not scale (measured 1.2x on 4 threads).

    Sized ONCE per process, by the first caller (the rank's configured worker count; chunk threads
    call this concurrently, creation happens under a lock): a later request for more workers gets
    the same pool, so no second pool ever oversubscribes the rank's pinned CPU slice and no pool
    is replaced while another thread may still be submitting to it."""
    global _PPOOL, _PPOOL_N
    with _PPOOL_LOCK:
        if _PPOOL is None:
            import multiprocessing as mp
            from concurrent.futures import ProcessPoolExecutor

            _PPOOL = ProcessPoolExecutor(max_workers=max(1, workers), mp_context=mp.get_context("spawn"))
            _PPOOL_N = workers
        return _PPOOL


def _partition_task(mlp, lo, hi, pa_idx, ra_idx, tau, values, pairs, rb, node_budget, limit, deadline, rbp=None):
    from ..engine import exact

    if deadline is not None:
        limit = min(limit, deadline - time.time())
        if limit <= 0.05:
            return "unknown", None, 0

    def confirm(xs, xps):
        ok = exact.check_pair_constraints(xs[None], xps[None], lo[None], hi[None], pa_idx, ra_idx, tau)
        return bool(ok[0] and exact.is_violation(mlp, xs[None], xps[None])[0])

    def exact_sign(xs):
        return int(exact.exact_signs(mlp, xs[None])[0])

    return solve_partition(mlp.weights, mlp.biases, lo, hi, pa_idx, values, pairs, rb, node_budget, limit, confirm,
                           exact_sign, ra_idx=ra_idx, tau=tau, row_bounds_p=rbp)


def submit(be, mlp, q, lo: np.ndarray, hi: np.ndarray, values: np.ndarray, pairs: np.ndarray, node_budget: int,
           time_limit: float, workers: int = 8, deadline: Optional[float] = None):
    """One future per partition -> (verdict, (x, x') or None, nodes).  Rigorous per-layer bounds
    come from the device in one launch (smt/milp.py:layer_bounds_rows); the LP-BaBs run in the
    worker processes.  ``deadline``: absolute time.time() after which nothing starts."""
    from . import milp

    if len(lo) == 0:
        return []
    lbs, ubs = milp.layer_bounds_rows(be, lo, hi, q, values, widen_ra=False)
    if q.relaxed:         # x' rows: RA dims widened by tau (unclipped, reference semantics)
        lbp, ubp = milp.layer_bounds_rows(be, lo, hi, q, values, widen_ra=True)
    V = values.shape[0]
    ex = process_pool(workers)
    futs = []
    for k in range(len(lo)):
        rb = {v: ([lb[k, v] for lb in lbs], [ub[k, v] for ub in ubs]) for v in range(V)}
        rbp = {v: ([lb[k, v] for lb in lbp], [ub[k, v] for ub in ubp]) for v in range(V)} if q.relaxed else None
        futs.append(ex.submit(_partition_task, mlp, lo[k], hi[k], tuple(q.pa_idx), tuple(q.ra_idx), float(q.tau),
                              values, pairs, rb, int(node_budget), float(time_limit), deadline, rbp))
    return futs
