"""Host MILP back-end for the residual partitions (HiGHS through ``scipy.optimize.milp``).

The reference decides every partition with Z3 over the exact network encoding
(utils/verif_utils.py, src/AC/Verify-AC.py:127-163).  Z3 is not in this image; HiGHS ships with
SciPy.  This back-end encodes the SAME fairness query as a mixed-integer program and is fed the
GPU's rigorous per-layer bounds (symbolic kernel, ``keep_layers``) as big-M constants, so only
neurons the GPU could not stabilise become binaries (the GPU-pruned subnetwork of SURVEY §3):

    for an ordered PA pair (v, v'):   maximise t
        x integer in the partition box, PA dims = v;  x' = x except PA = v' and, for relaxed
        attributes, |x'_r - x_r| <= tau;   t <= -N(x, v),  t <= N(x', v')
    every hidden neuron:  stable active  h = z;  stable inactive  h = 0;
                          unstable       h >= z, h >= 0, h <= z - lb (1 - a), h <= ub a, a binary.

``t* > 0`` iff a violating pair exists in that orientation.  Decision with a margin ``delta``
(default 1e-4 logit units, far above HiGHS's 1e-7 feasibility tolerance times the weight
magnitudes of the zoo networks):

* ``sat``   -- optimal t* > delta: the solution (x, x') is returned as a CANDIDATE; the pipeline
  confirms it with the exact rational checker before the partition counts as SAT;
* ``unsat`` -- every ordered pair's dual bound on t* is < -delta;
* ``unknown`` otherwise (time limit, or t* within the margin).

UNSAT from this stage rests on HiGHS's floating-point branch-and-cut (like the reference's
reliance on Z3); it is reported as its own stage (``milp``) in the CSV/JSON accounting.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

Result = Tuple[str, Optional[Tuple[List[int], List[int]]]]


def available() -> bool:
    try:
        from scipy.optimize import milp  # noqa: F401

        return True
    except Exception:
        return False


@dataclass
class _Builder:
    nv: int = 0

    def __post_init__(self):
        self.lb: List[float] = []
        self.ub: List[float] = []
        self.integ: List[int] = []
        self.r_i: List[np.ndarray] = []     # COO rows
        self.r_j: List[np.ndarray] = []
        self.r_v: List[np.ndarray] = []
        self.r_lo: List[np.ndarray] = []
        self.r_hi: List[np.ndarray] = []
        self.nr = 0

    def vars(self, lb, ub, integer=0) -> np.ndarray:
        lb = np.atleast_1d(np.asarray(lb, dtype=np.float64))
        ub = np.atleast_1d(np.asarray(ub, dtype=np.float64))
        k = lb.size
        idx = np.arange(self.nv, self.nv + k)
        self.nv += k
        self.lb.extend(lb.tolist())
        self.ub.extend(ub.tolist())
        self.integ.extend([integer] * k)
        return idx

    def rows(self, i_local: np.ndarray, j: np.ndarray, v: np.ndarray, lo: np.ndarray, hi: np.ndarray) -> None:
        """Rows with local indices 0..len(lo)-1 (appended after the existing rows)."""
        self.r_i.append(np.asarray(i_local, dtype=np.int64) + self.nr)
        self.r_j.append(np.asarray(j, dtype=np.int64))
        self.r_v.append(np.asarray(v, dtype=np.float64))
        self.r_lo.append(np.asarray(lo, dtype=np.float64))
        self.r_hi.append(np.asarray(hi, dtype=np.float64))
        self.nr += len(lo)


def _network(B: _Builder, weights: Sequence[np.ndarray], biases: Sequence[np.ndarray], x_idx: np.ndarray,
             x_const: np.ndarray, lbs: Sequence[np.ndarray], ubs: Sequence[np.ndarray]):
    """Encode one network copy.  Input dim d is variable ``x_idx[d]`` (>= 0) or the constant
    ``x_const[d]`` (x_idx[d] < 0).  Returns (output coefficient indices, values, constant)."""
    prev_idx = np.asarray(x_idx, dtype=np.int64)
    prev_const = np.asarray(x_const, dtype=np.float64)
    L = len(weights)
    for l in range(L - 1):
        W = np.asarray(weights[l], dtype=np.float64)
        b = np.asarray(biases[l], dtype=np.float64).copy()
        var = prev_idx >= 0
        # constant inputs fold into the bias
        if (~var).any():
            b = b + prev_const[~var] @ W[~var]
        Wv = W[var]                                     # [n_var_in, w]
        pin = prev_idx[var]
        lb = np.asarray(lbs[l], dtype=np.float64)
        ub = np.asarray(ubs[l], dtype=np.float64)
        w = W.shape[1]
        act = lb >= 0
        dead = ub <= 0
        unst = ~act & ~dead
        h = B.vars(np.zeros(w), np.where(dead, 0.0, np.maximum(ub, 0.0)))
        nin = pin.size
        # stable active: h_j - W_j . h_prev = b_j
        ja = np.nonzero(act)[0]
        if ja.size:
            k = ja.size
            ii = np.concatenate([np.arange(k), np.repeat(np.arange(k), nin)])
            jj = np.concatenate([h[ja], np.tile(pin, k)])
            vv = np.concatenate([np.ones(k), -Wv[:, ja].T.reshape(-1)])
            B.rows(ii, jj, vv, b[ja], b[ja])
        ju = np.nonzero(unst)[0]
        if ju.size:
            k = ju.size
            a = B.vars(np.zeros(k), np.ones(k), integer=1)
            base_i = np.concatenate([np.arange(k), np.repeat(np.arange(k), nin)])
            base_j = np.concatenate([h[ju], np.tile(pin, k)])
            base_v = np.concatenate([np.ones(k), -Wv[:, ju].T.reshape(-1)])
            # h - W.h_prev >= b
            B.rows(base_i, base_j, base_v, b[ju], np.full(k, np.inf))
            # h - W.h_prev - lb a <= b - lb
            B.rows(np.concatenate([base_i, np.arange(k)]), np.concatenate([base_j, a]),
                   np.concatenate([base_v, -lb[ju]]), np.full(k, -np.inf), b[ju] - lb[ju])
            # h - ub a <= 0
            B.rows(np.concatenate([np.arange(k), np.arange(k)]), np.concatenate([h[ju], a]),
                   np.concatenate([np.ones(k), -ub[ju]]), np.full(k, -np.inf), np.zeros(k))
        prev_idx = h
        prev_const = np.zeros(w)
    W = np.asarray(weights[-1], dtype=np.float64)[:, 0]
    b = float(np.asarray(biases[-1], dtype=np.float64)[0])
    var = prev_idx >= 0
    b += float(prev_const[~var] @ W[~var])
    return prev_idx[var], W[var], b


def solve_pair(weights, biases, lo: np.ndarray, hi: np.ndarray, pa_idx: Sequence[int], va: np.ndarray,
               vb: np.ndarray, ra_idx: Sequence[int], tau: float, bounds_a, bounds_b, time_limit: float,
               delta: float = 1e-4):
    """One ordered PA pair: returns (t_star or None, t_upper_bound, x, x') -- x/x' None if no
    primal solution was found."""
    from scipy.optimize import Bounds, LinearConstraint, milp
    from scipy.sparse import coo_matrix

    n0 = lo.size
    pa = list(pa_idx)
    ra = set(int(r) for r in ra_idx) if tau > 0 else set()
    B = _Builder()
    x_lb = lo.astype(np.float64).copy()
    x_ub = hi.astype(np.float64).copy()
    x_lb[pa] = va
    x_ub[pa] = va
    x = B.vars(x_lb, x_ub, integer=1)
    xa_idx = x.copy()
    xb_idx = x.copy()
    xb_const = np.zeros(n0)
    for k, d in enumerate(pa):
        xb_idx[d] = -1
        xb_const[d] = float(vb[k])
    rvars = {}
    for d in sorted(ra):
        v = B.vars([lo[d] - tau], [hi[d] + tau], integer=1)[0]
        rvars[d] = v
        xb_idx[d] = v
        # |x'_d - x_d| <= tau
        B.rows(np.array([0, 0]), np.array([v, x[d]]), np.array([1.0, -1.0]), np.array([-tau]), np.array([tau]))
    ia, wa, ba = _network(B, weights, biases, xa_idx, np.zeros(n0), *bounds_a)
    ib, wb, bb = _network(B, weights, biases, xb_idx, xb_const, *bounds_b)
    t = B.vars([-np.inf], [np.inf])[0]
    # t + N_A <= 0 ;  N_B - t >= 0
    B.rows(np.zeros(ia.size + 1, np.int64), np.concatenate([ia, [t]]), np.concatenate([wa, [1.0]]),
           np.array([-np.inf]), np.array([-ba]))
    B.rows(np.zeros(ib.size + 1, np.int64), np.concatenate([ib, [t]]), np.concatenate([wb, [-1.0]]),
           np.array([-bb]), np.array([np.inf]))
    c = np.zeros(B.nv)
    c[t] = -1.0
    A = coo_matrix((np.concatenate(B.r_v), (np.concatenate(B.r_i), np.concatenate(B.r_j))), shape=(B.nr, B.nv))
    res = milp(c, constraints=LinearConstraint(A.tocsr(), np.concatenate(B.r_lo), np.concatenate(B.r_hi)),
               integrality=np.asarray(B.integ), bounds=Bounds(np.asarray(B.lb), np.asarray(B.ub)),
               options=dict(time_limit=max(0.01, float(time_limit)), disp=False))
    t_star = None
    xs = xps = None
    if res.x is not None:
        t_star = -float(res.fun)
        xs = np.rint(res.x[x]).astype(np.int64)
        xps = xs.copy()
        for k, d in enumerate(pa):
            xps[d] = int(vb[k])
        for d, v in rvars.items():
            xps[d] = int(np.rint(res.x[v]))
    dual = getattr(res, "mip_dual_bound", None)
    if res.status == 2:                      # infeasible: no x at all (cannot happen with a box)
        return None, -np.inf, None, None
    # upper bound on t* = the solver's dual bound (the branch-and-bound's proven bound)
    t_ub = -float(dual) if dual is not None and np.isfinite(dual) else np.inf
    return t_star, t_ub, xs, xps


def output_bound(weights, biases, lo: np.ndarray, hi: np.ndarray, pa_idx: Sequence[int], va: np.ndarray, bounds,
                 sense: float, time_limit: float) -> float:
    """Proven bound of one network copy over the integer box with PA = va: a lower bound on
    min N (sense +1) or an upper bound on max N (sense -1), from the MILP's dual bound
    (-inf / +inf when nothing was proven in time).  Half the binaries of the pair query."""
    from scipy.optimize import Bounds, LinearConstraint, milp
    from scipy.sparse import coo_matrix

    pa = list(pa_idx)
    B = _Builder()
    x_lb = lo.astype(np.float64).copy()
    x_ub = hi.astype(np.float64).copy()
    x_lb[pa] = va
    x_ub[pa] = va
    x = B.vars(x_lb, x_ub, integer=1)
    io, wo, bo = _network(B, weights, biases, x, np.zeros(lo.size), *bounds)
    c = np.zeros(B.nv)
    c[io] = sense * wo
    if B.nr:
        A = coo_matrix((np.concatenate(B.r_v), (np.concatenate(B.r_i), np.concatenate(B.r_j))), shape=(B.nr, B.nv))
        cons = LinearConstraint(A.tocsr(), np.concatenate(B.r_lo), np.concatenate(B.r_hi))
    else:
        cons = ()
    res = milp(c, constraints=cons, integrality=np.asarray(B.integ), bounds=Bounds(np.asarray(B.lb), np.asarray(B.ub)),
               options=dict(time_limit=max(0.01, float(time_limit)), disp=False))
    dual = getattr(res, "mip_dual_bound", None)
    if dual is None or not np.isfinite(dual):
        return -np.inf * sense
    return sense * (float(dual) + sense * bo)


def solve_partition(weights, biases, lo: np.ndarray, hi: np.ndarray, pa_idx, values: np.ndarray, pairs: np.ndarray,
                    ra_idx, tau: float, row_bounds, xp_bounds, time_limit: float, delta: float = 1e-4) -> Result:
    """Decide one partition: ``row_bounds[v]`` / ``xp_bounds[v]`` = (per-layer lb list, ub list)
    of the x rows / x' rows with PA value index v.

    First the cheap sign test: if the network is provably positive (or negative) on every row
    of the partition, no pair can flip (single-copy MILPs, half the binaries); otherwise one
    pair MILP per ordered PA pair."""
    import time

    t_end = time.time() + time_limit
    V = len(values)
    rows = [(v, row_bounds[v], lo, hi) for v in range(V)]
    if tau > 0 and len(ra_idx):
        plo, phi = lo.astype(np.float64).copy(), hi.astype(np.float64).copy()
        for r in ra_idx:
            plo[r] -= tau
            phi[r] += tau
        rows += [(v, xp_bounds[v], plo, phi) for v in range(V)]
    for sense in (1.0, -1.0):
        proven = True
        for v, bnd, blo, bhi in rows:
            left = t_end - time.time()
            if left <= 0:
                return "unknown", None
            b = output_bound(weights, biases, blo, bhi, pa_idx, values[v], bnd, sense, left)
            if not (sense * b > delta):
                proven = False
                break
        if proven:
            return "unsat", None
    all_unsat = True
    for vi, vj in pairs:
        left = t_end - time.time()
        if left <= 0:
            return "unknown", None
        t_star, t_ub, xs, xps = solve_pair(weights, biases, lo, hi, pa_idx, values[vi], values[vj], ra_idx, tau,
                                           row_bounds[int(vi)], xp_bounds[int(vj)], left, delta)
        if t_star is not None and t_star > delta and xs is not None:
            return "sat", (xs.tolist(), xps.tolist())
        if not (t_ub < -delta):
            all_unsat = False
    return ("unsat", None) if all_unsat else ("unknown", None)


# ---------------------------------------------------------------------------------------------
_POOL = None


def pool(workers: int = 8):
    """Process-wide worker threads for the MILP stage (HiGHS releases the GIL while it solves)."""
    global _POOL
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor

        _POOL = ThreadPoolExecutor(max_workers=max(1, workers), thread_name_prefix="milp")
    return _POOL


def layer_bounds_rows(be, lo: np.ndarray, hi: np.ndarray, q, values: np.ndarray, widen_ra: bool):
    """Rigorous per-layer pre-activation bounds of every (partition, PA value) row on the device
    (symbolic kernel, keep_layers): returns lists ``lb[l]``, ``ub[l]`` of [P, V, w_l] arrays.
    ``widen_ra``: the x' rows of a relaxed query (RA dims widened by tau)."""
    import torch

    P, n = lo.shape
    V = values.shape[0]
    rlo = np.repeat(lo[:, None, :], V, axis=1).astype(np.float32)
    rhi = np.repeat(hi[:, None, :], V, axis=1).astype(np.float32)
    rlo[:, :, list(q.pa_idx)] = values[None].astype(np.float32)
    rhi[:, :, list(q.pa_idx)] = values[None].astype(np.float32)
    if widen_ra and q.relaxed:
        ra = list(q.ra_idx)
        rlo[:, :, ra] -= q.tau
        rhi[:, :, ra] += q.tau
    dev = be.device
    from ..engine.bab import BaBConfig, refine_on

    # deep nets: hidden-layer bounds tightened by back-substitution (csrc/refine.hip) -- the LP's
    # triangle relaxation is only as tight as these intervals
    rf = refine_on(BaBConfig().refine, be.widths)
    res = be.bounds(torch.from_numpy(rlo.reshape(P * V, n)).to(dev), torch.from_numpy(rhi.reshape(P * V, n)).to(dev),
                    mode="symbolic", keep_layers=True, crown=rf, refine=rf)
    # every layer's [lb | ub] rows packed on the device, ONE async copy into pinned host memory on a
    # side stream (the north star's pinned hipMemcpyAsync feed of the host solver) instead of 2L
    # blocking .cpu() copies
    parts = [t.float() for t in res.layer_lb] + [t.float() for t in res.layer_ub]
    packed = torch.cat(parts, dim=1)
    if packed.device.type == "cuda":
        host = torch.empty(packed.shape, dtype=torch.float32, pin_memory=True)
        side = _side_stream(packed.device)
        side.wait_stream(torch.cuda.current_stream(packed.device))
        with torch.cuda.stream(side):
            host.copy_(packed, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(side)
        packed.record_stream(side)
        ev.synchronize()
        hp = host.numpy()
    else:
        hp = packed.numpy()
    widths = [t.shape[1] for t in parts]
    offs = np.concatenate([[0], np.cumsum(widths)])
    cols = [hp[:, offs[i]:offs[i + 1]].reshape(P, V, -1).astype(np.float64) for i in range(len(parts))]
    L = len(res.layer_lb)
    return cols[:L], cols[L:]


_SIDE = {}


def _side_stream(dev):
    """One side stream per (device, host thread) for the bounds copy to the host solver."""
    import threading

    import torch

    k = (dev.index or 0, threading.get_ident())
    if k not in _SIDE:
        _SIDE[k] = torch.cuda.Stream(dev)
    return _SIDE[k]


def submit(be, mlp, q, lo: np.ndarray, hi: np.ndarray, values: np.ndarray, pairs: np.ndarray, time_limit: float,
           workers: int = 8, delta: float = 1e-4, deadline: Optional[float] = None):
    """One future per partition -> (verdict, (x, x') or None).  Bounds are computed on the device
    first (one launch for all rows), the MILPs then run on the host worker threads.  Each
    partition gets ``time_limit`` seconds, cut to what is left before the absolute ``deadline``
    (``time.time()`` scale); partitions whose turn comes after the deadline stay UNKNOWN."""
    import time as _time

    if len(lo) == 0:
        return []
    lbs, ubs = layer_bounds_rows(be, lo, hi, q, values, widen_ra=False)
    if q.relaxed:
        plbs, pubs = layer_bounds_rows(be, lo, hi, q, values, widen_ra=True)
    else:
        plbs, pubs = lbs, ubs
    V = values.shape[0]
    W, b = mlp.weights, mlp.biases

    def work(k: int):
        limit = time_limit
        if deadline is not None:
            limit = min(limit, deadline - _time.time())
            if limit <= 0.05:
                return "unknown", None
        rb = {v: ([lb[k, v] for lb in lbs[:-1]] + [lbs[-1][k, v]], [ub[k, v] for ub in ubs[:-1]] + [ubs[-1][k, v]])
              for v in range(V)}
        pb = {v: ([lb[k, v] for lb in plbs[:-1]] + [plbs[-1][k, v]], [ub[k, v] for ub in pubs[:-1]] + [pubs[-1][k, v]])
              for v in range(V)}
        return solve_partition(W, b, lo[k], hi[k], q.pa_idx, values, pairs, q.ra_idx, float(q.tau), rb, pb,
                               limit, delta)

    ex = pool(workers)
    return [ex.submit(work, k) for k in range(len(lo))]
