"""beta-CROWN ReLU-phase branch-and-bound (stage ``beta``; bounding in ops/beta.py, csrc/beta.hip).

The residue of the wide, deep networks (trained AC-7: 64-32-16-8-4) is what the input-split BaB
(engine/bab.py) and the interval-clamping ReLU-phase stage (engine/relu_bab.py) leave: its UNSAT
partitions need ReLU case splits that act as constraints on the input region, which is how Z3
decides them in the reference (utils/verif_utils.py:525-528, src/AC/Verify-AC.py:146-158) and how
the host verified LP (smt/lpbab.py) does, at ~2 s per partition per CPU worker.  Here every node
(partition, ordered PA pair, box, phases of both copies) is bounded on the GPU by the
Lagrangian (beta) bound of ops/beta.py with optimised slopes / split multipliers, warm-started from
its parent; a rigorous fp64 re-evaluation decides.

Search: one tree per (partition, ordered PA pair) in a FIFO node pool processed in batches (the
first batch of roots with ``root_iters`` optimisation steps, the rest with ``iters``); a node
closes when its bound is >= 0 (no pair with N(x, va) < 0 < N(x, vb) in its region: f_t < 0 on any
such pair), its concretising vertex pair is screened with rigorous point bounds and confirmed exactly
on the host (SAT), a single lattice point is decided exactly, and a partition whose nodes all
closed is UNSAT.  A partition past its node budget ends UNKNOWN.

PA-only queries (relaxed queries keep the relu / LP stages).  CPU tests pin verdicts to brute-force
enumeration (tests/test_beta_bab.py); the GPU kernel to this module's reference (tests/test_beta_gpu.py).
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from ..models.mlp import MLP
from ..ops import beta as B
from ..ops.backend import Backend
from ..spec import ResolvedQuery
from ..utils.timer import NULL, StageTimer
from . import exact
from .bab import RUNNING, SAT, UNKNOWN, UNSAT, BaBResult, _pa_table, pa_groups


@dataclass
class BetaConfig:
    node_budget: int = 512           # nodes per partition (all its pair trees together)
    iters: int = 64                  # optimisation steps per node (warm-started from the parent)
    root_iters: int = 200            # ... per root node
    lr_a: float = 0.1                # Adam step of the slopes alpha
    lr_b: float = 0.5                # ... of the split multipliers beta
    lr_t: float = 0.1                # ... of the pair weight t
    child_lr: float = 0.3            # children (warm-started at their parent's optimum): lr x this
    decay: float = 0.98              # lr decay per step
    warm_beta: bool = True           # split multiplier starts at the parent's relaxation (else 0)
    cold: bool = False               # children: also optimise from the cold start, keep the better
    lookahead: int = 8               # filtered branching: candidates per score (0 = best gap score)
    beta_pos: bool = True            # split multipliers projected >= 0 (free-signed ones, which may
    #                                  use the interval side, make Adam oscillate around 0: measured
    #                                  8 / 10 -> 0 / 10 trained AC-7 partitions closed, tools/exp)
    batch_nodes: int = 32768         # nodes per level launch
    time_budget: float = 1e9         # wall-clock seconds for the whole call
    max_pool: int = 1 << 21          # live nodes (more: the partitions losing nodes end UNKNOWN)


def supported(q: ResolvedQuery) -> bool:
    return not q.relaxed


def fits(be: Backend) -> bool:
    """The kernel's shape limits (inputs <= 64, weights within LDS); the torch reference has none."""
    if not be.hip:
        return True
    from ..ops import ext
    from ..ops.hip import _net

    return bool(ext().beta_fits(_net(be)))


class BetaBaBSolver:
    def __init__(self, backend: Backend, query: ResolvedQuery, cfg: BetaConfig, timer: StageTimer = NULL):
        self.be = backend
        self.q = query
        self.cfg = cfg
        self.tm = timer
        self.dev = backend.device
        self.stats = {}

    def solve(self, lo_np: np.ndarray, hi_np: np.ndarray, mlp_exact: MLP,
              init_status: Optional[np.ndarray] = None) -> BaBResult:
        t0 = time.time()
        P, n = lo_np.shape
        status = np.full(P, RUNNING, dtype=np.int8) if init_status is None else init_status.astype(np.int8).copy()
        cex_x = np.zeros((P, n), dtype=np.int64)
        cex_xp = np.zeros((P, n), dtype=np.int64)
        nodes = np.zeros(P, dtype=np.int64)
        if not supported(self.q) or self.be.n_hidden == 0 or not fits(self.be):
            status[status == RUNNING] = UNKNOWN
            return BaBResult(status, cex_x, cex_xp, nodes)
        self.stats = {"levels": 0, "nodes": 0}
        for g in pa_groups(self.q, lo_np, hi_np):
            left = max(0.0, self.cfg.time_budget - (time.time() - t0))
            st, cx, cxp, nd = self._solve_group(lo_np[g], hi_np[g], mlp_exact, status[g], left)
            status[g], cex_x[g], cex_xp[g], nodes[g] = st, cx, cxp, nd
        return BaBResult(status, cex_x, cex_xp, nodes, 0, time.time() - t0)

    # ------------------------------------------------------------------------------------------
    def _root_bounds(self, lo: torch.Tensor, hi: torch.Tensor, values: torch.Tensor):
        """Rigorous per-layer pre-activation bounds [P * V, NH] of every (partition, PA value) row
        (the verified LP's bounds, smt/milp.py:layer_bounds_rows, kept on the device)."""
        be, q = self.be, self.q
        P, n0 = lo.shape
        V = values.shape[0]
        pa = list(q.pa_idx)
        rlo = lo.repeat_interleave(V, dim=0)
        rhi = hi.repeat_interleave(V, dim=0)
        vv = values.repeat(P, 1)
        rlo[:, pa] = vv
        rhi[:, pa] = vv
        rf = len(be.widths) - 1 >= 2        # refined hidden bounds: every relaxation above layer 0 tightens
        res = be.bounds(rlo, rhi, mode="symbolic", keep_layers=True, crown=rf, refine=rf)
        NH = be.n_hidden
        lb = torch.cat([t.float() for t in res.layer_lb], 1)[:, :NH].contiguous()
        ub = torch.cat([t.float() for t in res.layer_ub], 1)[:, :NH].contiguous()
        return lb, ub

    def _solve_group(self, lo_np, hi_np, mlp_exact, status, time_budget):
        t0 = time.time()
        be, q, cfg = self.be, self.q, self.cfg
        dev = self.dev
        P, n0 = lo_np.shape
        NH = be.n_hidden
        status = status.copy()
        cex_x = np.zeros((P, n0), dtype=np.int64)
        cex_xp = np.zeros((P, n0), dtype=np.int64)
        nodes_np = np.zeros(P, dtype=np.int64)
        values_np, pairs_np = _pa_table(q, lo_np, hi_np)
        run = np.nonzero(status == RUNNING)[0]
        Pp = pairs_np.shape[0]
        if Pp == 0:
            status[run] = UNSAT
            return status, cex_x, cex_xp, nodes_np
        if run.size == 0:
            return status, cex_x, cex_xp, nodes_np
        pa = list(q.pa_idx)
        f32 = dict(dtype=torch.float32, device=dev)
        values = torch.from_numpy(values_np.astype(np.float32)).to(dev)
        V = values.shape[0]
        lo_r = torch.from_numpy(lo_np[run].astype(np.float32)).to(dev)
        hi_r = torch.from_numpy(hi_np[run].astype(np.float32)).to(dev)
        with self.tm("beta.roots"):
            rlb, rub = self._root_bounds(lo_r, hi_r, values)
        # one root per (running partition, ordered pair)
        k = torch.arange(run.size, device=dev).repeat_interleave(Pp)
        pr = torch.from_numpy(pairs_np.astype(np.int64)).to(dev).repeat(run.size, 1)
        ra, rb = k * V + pr[:, 0], k * V + pr[:, 1]
        pool = {
            "part": torch.from_numpy(run).to(dev)[k],
            "lo": lo_r[k].clone(), "hi": hi_r[k].clone(),
            "va": values[pr[:, 0]].clone(), "vb": values[pr[:, 1]].clone(),
            "LBA": rlb[ra], "UBA": rub[ra], "LBB": rlb[rb], "UBB": rub[rb],
            "phA": torch.zeros(k.numel(), NH, dtype=torch.int8, device=dev),
            "phB": torch.zeros(k.numel(), NH, dtype=torch.int8, device=dev),
            "alA": torch.full((k.numel(), NH), 0.5, **f32), "alB": torch.full((k.numel(), NH), 0.5, **f32),
            "beA": torch.zeros(k.numel(), NH, **f32), "beB": torch.zeros(k.numel(), NH, **f32),
            "t": torch.full((k.numel(),), 0.5, **f32),
            "root": torch.ones(k.numel(), dtype=torch.bool, device=dev),
        }
        free = torch.ones(n0, dtype=torch.bool, device=dev)
        free[pa] = False
        levels = 0
        timed_out = False
        while pool["part"].numel():
            if time.time() - t0 > time_budget:
                timed_out = True
                break
            # drop nodes of decided / over-budget partitions
            alive = torch.from_numpy(status == RUNNING).to(dev)[pool["part"]]
            if not bool(alive.all()):
                pool = {kk: v[alive] for kk, v in pool.items()}
                if not pool["part"].numel():
                    break
            # the front batch: roots first (their own iteration count), then FIFO
            nb = min(cfg.batch_nodes, pool["part"].numel())
            is_root = bool(pool["root"][0])
            if is_root:
                nb = min(nb, int(pool["root"].sum()))
            cur = {kk: v[:nb] for kk, v in pool.items()}
            rest = {kk: v[nb:] for kk, v in pool.items()}
            levels += 1
            part_np = cur["part"].cpu().numpy()
            np.add.at(nodes_np, part_np, 1)
            sc = 1.0 if is_root else cfg.child_lr
            with self.tm("beta.level"):
                lev = be.beta_level(cur["lo"], cur["hi"], pa, cur["va"], cur["vb"], cur["LBA"], cur["UBA"],
                                    cur["LBB"], cur["UBB"], cur["phA"], cur["phB"], cur["alA"], cur["alB"],
                                    cur["beA"], cur["beB"], cur["t"], cfg.root_iters if is_root else cfg.iters,
                                    cfg.lr_a * sc, cfg.lr_b * sc, cfg.lr_t * sc, cfg.decay, cfg.lookahead, cfg.beta_pos)
            if cfg.cold and not is_root:
                c2 = {kk: cur[kk].clone() for kk in ("alA", "alB", "beA", "beB", "t")}
                c2["alA"].fill_(0.5); c2["alB"].fill_(0.5); c2["beA"].zero_(); c2["beB"].zero_(); c2["t"].fill_(0.5)
                lev2 = be.beta_level(cur["lo"], cur["hi"], pa, cur["va"], cur["vb"], cur["LBA"], cur["UBA"],
                                     cur["LBB"], cur["UBB"], cur["phA"], cur["phB"], c2["alA"], c2["alB"],
                                     c2["beA"], c2["beB"], c2["t"], cfg.root_iters, cfg.lr_a, cfg.lr_b, cfg.lr_t,
                                     cfg.decay, cfg.lookahead, cfg.beta_pos)
                use = lev2.bound > lev.bound
                for kk in c2:
                    cur[kk][use] = c2[kk][use]
                lev = B.BetaLevel(bound=torch.where(use, lev2.bound, lev.bound),
                                  split=torch.where(use, lev2.split, lev.split),
                                  xstar=torch.where(use[:, None], lev2.xstar, lev.xstar),
                                  binit=torch.where(use[:, None], lev2.binit, lev.binit))
            closed = lev.bound >= 0
            leaf = lev.split == -(n0 + 1)
            # candidate vertex pairs of the nodes that stay open (and the lattice leaves): rigorous
            # point bounds screen, then the exact check on the host
            cand = torch.nonzero(~closed).flatten()
            if cand.numel():
                xa = lev.xstar[cand].clone()
                xb = xa.clone()
                xa[:, pa] = cur["va"][cand]
                xb[:, pa] = cur["vb"][cand]
                with self.tm("beta.cand"):
                    alb, _ = be.point_bounds(xa)
                    _, bub = be.point_bounds(xb)
                poss = (alb < 0) & (bub > 0)
                ci = cand[poss]
                if ci.numel():
                    self._confirm(cur["part"][ci].cpu().numpy(), xa[poss], xb[poss], status, cex_x, cex_xp,
                                  mlp_exact, lo_np, hi_np)
            grow = ~closed & ~leaf
            run_t = torch.from_numpy(status == RUNNING).to(dev)[cur["part"]]
            grow &= run_t
            over = torch.from_numpy(nodes_np >= cfg.node_budget).to(dev)[cur["part"]] & grow
            if bool(over.any()):
                status[np.unique(cur["part"][over].cpu().numpy())] = UNKNOWN
                grow &= ~over
            gi = torch.nonzero(grow).flatten()
            bi = lev.binit[gi] if cfg.warm_beta else torch.zeros_like(lev.binit[gi])
            kids = self._children({kk: v[gi] for kk, v in cur.items()}, lev.split[gi], bi, NH, n0)
            pool = {kk: torch.cat([rest[kk], kids[kk]]) for kk in pool}
            if pool["part"].numel() > cfg.max_pool:
                lost = torch.unique(pool["part"][cfg.max_pool:]).cpu().numpy()
                status[lost[status[lost] == RUNNING]] = UNKNOWN
                pool = {kk: v[:cfg.max_pool] for kk, v in pool.items()}
        left = set(pool["part"].cpu().numpy().tolist()) if (timed_out and pool["part"].numel()) else set()
        for p in np.nonzero(status == RUNNING)[0]:
            status[p] = UNKNOWN if p in left else UNSAT
        self.stats["levels"] = self.stats.get("levels", 0) + levels
        self.stats["nodes"] = self.stats.get("nodes", 0) + int(nodes_np.sum())
        return status, cex_x, cex_xp, nodes_np

    @staticmethod
    def _children(nd, split, binit, NH: int, n0: int):
        """Two children per node: a phase split (split >= 0: copy A neuron split, copy B NH + j)
        inheriting the parent's parameters (the new multiplier from ``binit``: the child starts at
        the parent's bound), or an input split
        (split = -1 - d) halving dim d."""
        R = split.numel()
        dev = split.device
        rep = torch.arange(R, device=dev).repeat_interleave(2)
        kid = {kk: v[rep].clone() for kk, v in nd.items()}
        kid["root"][:] = False
        if R == 0:
            return kid
        sp = split[rep]
        side = torch.arange(2 * R, device=dev) % 2             # 0: lower child, 1: upper child
        r_ = torch.arange(2 * R, device=dev)
        neu = sp >= 0
        sgn = torch.where(side == 0, -1, 1).to(torch.int8)
        inA = neu & (sp < NH)
        inB = neu & (sp >= NH)
        bi = binit[rep].gather(1, side[:, None])[:, 0]
        if bool(inA.any()):
            kid["phA"][r_[inA], sp[inA]] = sgn[inA]
            kid["beA"][r_[inA], sp[inA]] = bi[inA]
        if bool(inB.any()):
            kid["phB"][r_[inB], sp[inB] - NH] = sgn[inB]
            kid["beB"][r_[inB], sp[inB] - NH] = bi[inB]
        inp = ~neu
        if bool(inp.any()):
            d = (-1 - sp[inp]).clamp(0, n0 - 1)
            ri = r_[inp]
            lo_d = kid["lo"][ri, d]
            hi_d = kid["hi"][ri, d]
            mid = torch.floor((lo_d + hi_d) / 2)
            low_child = side[inp] == 0
            kid["hi"][ri[low_child], d[low_child]] = mid[low_child]
            kid["lo"][ri[~low_child], d[~low_child]] = mid[~low_child] + 1
        return kid

    def _confirm(self, parts, xa, xb, status, cex_x, cex_xp, mlp_exact, lo_np, hi_np):
        X = xa.cpu().numpy().round().astype(np.int64)
        XP = xb.cpu().numpy().round().astype(np.int64)
        ok = exact.check_pair_constraints(X, XP, lo_np[parts], hi_np[parts], self.q.pa_idx, self.q.ra_idx, self.q.tau)
        viol = exact.is_violation(mlp_exact, X, XP) & ok
        order = np.lexsort(tuple(np.concatenate([X, XP], axis=1).T[::-1]) + (parts,))
        for k in order:
            p = parts[k]
            if viol[k] and status[p] != SAT:
                status[p] = SAT
                cex_x[p], cex_xp[p] = X[k], XP[k]
