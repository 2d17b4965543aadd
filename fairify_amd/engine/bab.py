"""Batched branch-and-bound decision procedure for the fairness query (K8 + K9).

The reference decides a partition with one Z3 ``check()`` under a soft timeout
(src/AC/Verify-AC.py:127-163).  Z3 is not part of this framework; instead every partition of a
chunk is decided *together* by a device-resident branch-and-bound over the integer lattice:

* a node is an integer sub-box of the partition (plus, for relaxed attributes, a box for x');
* its rows (one per protected-attribute assignment v) are bounded with the symbolic bound
  propagation kernel, and :func:`pair_certify` proves "no violating pair inside" (node closed)
  or returns the most violating pair, a split dimension and a candidate vertex pair;
* candidates are evaluated with the fp32 forward + rounding bound and confirmed exactly on the
  host (``engine.exact``), so SAT answers are true counterexamples;
* leaves are single lattice points, evaluated exactly — the procedure is complete on the finite
  domain, budgets (nodes per partition, wall clock) turn the remainder into UNKNOWN.

All node bookkeeping is tensor code on the device; the only host round trip per iteration is
the (tiny) SAT-candidate list.
"""
from __future__ import annotations

import os
import threading
import time
from dataclasses import dataclass, field, replace
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..models.mlp import MLP
from ..ops.backend import Backend
from ..spec import ResolvedQuery
from ..utils.timer import NULL, StageTimer
from . import exact

UNKNOWN, SAT, UNSAT, RUNNING = 0, 1, 2, 3

# process-wide native-runtime counters (diagnostics: tools/diag_shard_diff.py, bench --profile)
STATS: Dict[str, int] = {"levels": 0, "launches": 0, "cand_overflow_levels": 0}
_STATS_LOCK = threading.Lock()
VERDICT_NAMES = {UNKNOWN: "unknown", SAT: "sat", UNSAT: "unsat", RUNNING: "running"}


@dataclass
class BaBConfig:
    node_budget: int = 4096          # max node expansions per partition (soft-timeout analogue)
    batch_nodes: int = 32768         # nodes bounded per iteration
    max_pool: int = 1 << 24          # live-node capacity per runtime (grown lazily; UNKNOWN beyond)
    time_budget: float = 1e9         # wall-clock seconds for the whole call
    mode: str = "symbolic"
    cand_cap: int = 1 << 17          # candidate pairs confirmed per BFS level (native runtime)
    crown: bool = os.environ.get("FAIRIFY_CROWN", "1") != "0"   # backward output bounds per node
    # hidden-layer bounds tightened by back-substitution before the output pass (csrc/refine.hip):
    # "auto" = networks with >= 3 hidden layers of which one is >= 10 wide (AC-7's residue closes
    # in ~800 nodes instead of > 32 768; on 1-2 hidden layers it equals the forward bounds), "on", "off"
    refine: str = os.environ.get("FAIRIFY_REFINE", "auto")
    # native runtime input-split scores: "auto" = first-layer smear (CertArgs.smear) for networks
    # whose first hidden layer is >= 32 wide (AC-2/3/4/5/7; the narrow deep nets keep the
    # certificate scores), "on", "off"
    smear: str = os.environ.get("FAIRIFY_SMEAR", "auto")
    # native runtime: the level end (fa_settle) runs in the level's last split launch (its last
    # workgroup) instead of its own launch.  Off: the device-scope release fence every workgroup
    # needs before counting itself done writes back the XCD's L2 (the level's children pool), and
    # cost more than the launch it saves (N=1 944 -> 1 011 ms/step, 1/8 shard 141 -> 169 ms,
    # profiles/r4/ab_fuse_settle.md)
    fuse_settle: bool = os.environ.get("FAIRIFY_FUSE_SETTLE", "0") == "1"
    # native runtime branching rule: a partition with w nodes in a BFS level splits each along
    # clamp(log2(split_target / w), 1, 6) dims (per partition: verdicts do not depend on which
    # partitions share a chunk)
    split_target: int = int(os.environ.get("FAIRIFY_SPLIT_TARGET", "256"))
    # native runtime inline escalation: a partition that reaches node_budget with a frontier of at
    # most escalate_max_w nodes continues up to escalate_budget (0 = off)
    escalate_budget: int = 0
    escalate_max_w: int = 0
    # intermediate (budget, max frontier) steps of the inline escalation, between node_budget and
    # escalate_budget: a partition continues past step k's budget only with a frontier of at most
    # its limit (fa_settle_kernel)
    escalate_steps: Tuple[Tuple[int, int], ...] = ()


@dataclass
class BaBResult:
    status: np.ndarray               # [P] int8 verdicts
    cex_x: np.ndarray                # [P, n0] int64 (valid where SAT)
    cex_xp: np.ndarray
    nodes: np.ndarray                # [P] int64 nodes expanded
    iters: int = 0
    time: float = 0.0
    open_left: Optional[np.ndarray] = None   # [P] open nodes left when an UNKNOWN partition stopped
                                             # (native runtime; the escalation filter's predictor)


def refine_level(mode: str, widths) -> int:
    """How the BaB bounds its nodes (BaBConfig.refine): 0 forward symbolic + backward output pass,
    1 with back-substituted hidden-layer bounds between them (csrc/refine.hip), 2 back-substitution
    alone (one launch, no forward pass).  ``auto``: level 1 for networks with at least 3 hidden
    layers, one of them at least 10 wide -- with 1-2 hidden layers the refined bounds equal the
    forward ones, and on the narrow deep nets (AC-9/10/12, 3-5 wide) the extra pass costs more than
    it closes (tools/diag_open_nodes.py on the bench residue)."""
    if mode in ("on", "refine"):
        return 1
    if mode == "full":
        return 2
    if mode != "auto":
        return 0
    hidden = list(widths)[:-1]
    return 1 if (len(hidden) >= 3 and max(hidden) >= 10) else 0


def smear_on(mode: str, widths) -> bool:
    """First-layer smear split scores in the native runtime (BaBConfig.smear)."""
    if mode == "on":
        return True
    if mode != "auto":
        return False
    return len(widths) >= 2 and int(widths[0]) >= 32


def refine_on(mode: str, widths) -> bool:
    """Hidden-layer bounds tightened by back-substitution (any level > 0 of :func:`refine_level`)."""
    return refine_level(mode, widths) > 0


def pa_groups(q: ResolvedQuery, lo: np.ndarray, hi: np.ndarray) -> List[np.ndarray]:
    """Row indices of the partitions sharing one protected-attribute range (one group when the
    chunk's PA ranges are identical, e.g. a PA that the partition size does not split)."""
    pa = list(q.pa_idx)
    if len(lo) == 0 or (np.all(lo[:, pa] == lo[:1, pa]) and np.all(hi[:, pa] == hi[:1, pa])):
        return [np.arange(len(lo))]
    key = np.concatenate([lo[:, pa], hi[:, pa]], axis=1)
    _, inv = np.unique(key, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    return [np.nonzero(inv == g)[0] for g in range(int(inv.max()) + 1)]


def _pa_table(q: ResolvedQuery, lo: np.ndarray, hi: np.ndarray):
    """PA assignments shared by all partitions of one PA group (:func:`pa_groups`)."""
    pa = list(q.pa_idx)
    assert np.all(lo[:, pa] == lo[:1, pa]) and np.all(hi[:, pa] == hi[:1, pa]), \
        "internal: one PA table per group (callers split with pa_groups)"
    values = q.pa_values(lo[0], hi[0])
    pairs = q.pa_pairs(values)
    return values, pairs


class BaBSolver:
    def __init__(self, backend: Backend, query: ResolvedQuery, cfg: BaBConfig, dead: Optional[torch.Tensor] = None,
                 timer: StageTimer = NULL):
        self.tm = timer
        self.be = backend
        self.q = query
        self.cfg = cfg
        self.dev = backend.device
        self.dead = dead            # optional [P, N_hidden] bool (heuristically pruned nets)
        n = query.n
        self.pa = torch.tensor(list(query.pa_idx), dtype=torch.long, device=self.dev)
        self.ra = torch.tensor(list(query.ra_idx), dtype=torch.long, device=self.dev)
        shared = np.ones(n, dtype=bool)
        shared[list(query.ra_idx)] = False
        self.shared = torch.from_numpy(shared).to(self.dev)     # PA dims are fixed per row -> "shared" ok
        self.relaxed = query.relaxed
        self.tau = float(query.tau)
        # mlp with dead-masks applied host-side for exact checks (per partition if masked)

    # --------------------------------------------------------------------------------------
    def _rows(self, lo: torch.Tensor, hi: torch.Tensor, values: torch.Tensor):
        """Expand node boxes [N, n] into node-major rows [N*V, n] with PA dims set to v."""
        N, n = lo.shape
        V = values.shape[0]
        rlo = lo[:, None, :].expand(N, V, n).clone()
        rhi = hi[:, None, :].expand(N, V, n).clone()
        vv = values.to(lo.dtype)[None, :, :].expand(N, V, values.shape[1])
        rlo[:, :, self.pa] = vv
        rhi[:, :, self.pa] = vv
        return rlo.reshape(N * V, n), rhi.reshape(N * V, n)

    def _eval_pairs(self, x: torch.Tensor, xp: torch.Tensor, part: torch.Tensor):
        """Rigorous evaluation of point pairs (value + running error bound that keeps exact
        zeros exact): returns (certain_violation, possible_but_uncertain) masks."""
        d = self.dead[part] if self.dead is not None else None
        xlb, xub = self.be.point_bounds(x, d)
        plb, pub = self.be.point_bounds(xp, d)
        sure = ((xub < 0) & (plb > 0)) | ((xlb > 0) & (pub < 0))
        poss = ((xlb < 0) & (pub > 0)) | ((xub > 0) & (plb < 0))
        return sure, poss & ~sure

    # --------------------------------------------------------------------------------------
    def solve(self, lo_np: np.ndarray, hi_np: np.ndarray, mlp_exact: MLP,
              init_status: Optional[np.ndarray] = None,
              exact_models: Optional[List[MLP]] = None) -> BaBResult:
        """Decide every partition box ``[lo_np[p], hi_np[p]]``.

        ``mlp_exact`` is the network used for exact confirmation (per-partition nets in
        ``exact_models`` when heuristic masks are active).
        """
        t0 = time.time()
        groups = pa_groups(self.q, lo_np, hi_np)
        if len(groups) > 1:
            return self._solve_groups(groups, lo_np, hi_np, mlp_exact, init_status, exact_models, t0)
        cfg = self.cfg
        dev = self.dev
        P, n = lo_np.shape
        values_np, pairs_np = _pa_table(self.q, lo_np, hi_np)
        values = torch.from_numpy(values_np).to(dev)
        pairs = torch.from_numpy(pairs_np).to(dev)
        V = values.shape[0]
        status = np.full(P, RUNNING, dtype=np.int8) if init_status is None else init_status.astype(np.int8).copy()
        cex_x = np.zeros((P, n), dtype=np.int64)
        cex_xp = np.zeros((P, n), dtype=np.int64)
        nodes_np = np.zeros(P, dtype=np.int64)
        if pairs.shape[0] == 0:
            status[status == RUNNING] = UNSAT   # a single PA value: no x' can differ
            return BaBResult(status, cex_x, cex_xp, nodes_np, 0, time.time() - t0)
        if self.be.hip and os.environ.get("FAIRIFY_TORCH_BAB") != "1":
            return self._solve_native(lo_np, hi_np, status, values_np, pairs_np, mlp_exact, exact_models, t0)

        dt = torch.float32
        run_idx = np.nonzero(status == RUNNING)[0]
        xlo = torch.from_numpy(lo_np[run_idx]).to(dev, dt)
        xhi = torch.from_numpy(hi_np[run_idx]).to(dev, dt)
        part = torch.from_numpy(run_idx).to(dev)
        if self.relaxed:
            xplo = xlo.clone()
            xphi = xhi.clone()
            xplo[:, self.ra] -= self.tau
            xphi[:, self.ra] += self.tau
        else:
            xplo, xphi = xlo, xhi
        status_t = torch.from_numpy(status).to(dev)
        nodes_t = torch.zeros(P, dtype=torch.long, device=dev)
        it = 0
        while xlo.shape[0] > 0:
            if time.time() - t0 > cfg.time_budget:
                break
            it += 1
            B = min(cfg.batch_nodes, xlo.shape[0])
            blo, bhi, bpart = xlo[:B], xhi[:B], part[:B]
            bplo, bphi = (xplo[:B], xphi[:B]) if self.relaxed else (blo, bhi)
            # drop nodes of partitions that are already decided
            alive = status_t[bpart] == RUNNING
            if not bool(alive.all()):
                blo, bhi, bpart, bplo, bphi = blo[alive], bhi[alive], bpart[alive], bplo[alive], bphi[alive]
            rest = slice(B, None)
            if blo.shape[0] == 0:
                xlo, xhi, part = xlo[rest], xhi[rest], part[rest]
                if self.relaxed:
                    xplo, xphi = xplo[rest], xphi[rest]
                continue
            Nn = blo.shape[0]
            nodes_t.index_add_(0, bpart, torch.ones_like(bpart))
            dead_rows = None
            if self.dead is not None:
                dead_rows = self.dead[bpart].repeat_interleave(V, dim=0)
            with self.tm("bab.bounds"):
                rlo, rhi = self._rows(blo, bhi, values)
                rf = refine_on(self.cfg.refine, self.be.widths)
                res_x = self.be.bounds(rlo, rhi, mode=cfg.mode, dead=dead_rows, crown=cfg.crown, refine=rf)
                if self.relaxed:
                    plo, phi = self._rows(bplo, bphi, values)
                    res_xp = self.be.bounds(plo, phi, mode=cfg.mode, dead=dead_rows, crown=cfg.crown, refine=rf)
                else:
                    res_xp = res_x
            with self.tm("bab.certify"):
                dec = self.be.pair_certify(res_x, res_xp, blo, bhi, bplo, bphi, pairs, values, self.pa, self.shared,
                                           self.relaxed)
            open_ = dec.open_
            # ---- candidate vertex pairs (falsification inside BaB)
            pv = pairs[dec.cand_v]
            cx = dec.cand_x.clone()
            cxp = dec.cand_xp.clone()
            cx[:, self.pa] = values[pv[:, 0]].to(cx.dtype)
            cxp[:, self.pa] = values[pv[:, 1]].to(cx.dtype)
            if self.relaxed:
                r = self.ra
                cxp[:, r] = torch.minimum(torch.maximum(cxp[:, r], cx[:, r] - self.tau), cx[:, r] + self.tau)
                cxp[:, r] = torch.minimum(torch.maximum(cxp[:, r], bplo[:, r]), bphi[:, r])
            # ---- leaves: single lattice points (x and x'); evaluate every pair exactly
            wmask = torch.ones(blo.shape[1], dtype=torch.bool, device=blo.device)
            wmask[self.pa] = False
            width = (bhi - blo)[:, wmask].amax(dim=1)
            if self.relaxed:
                width = torch.maximum(width, (bphi - bplo)[:, self.ra].amax(dim=1) if self.ra.numel() else width)
            leaf = open_ & (width == 0)
            sel = open_ & (status_t[bpart] == RUNNING)
            cand_rows = torch.nonzero(sel & ~leaf).flatten()
            found_idx: List[int] = []
            found_x: List[np.ndarray] = []
            found_xp: List[np.ndarray] = []
            if cand_rows.numel():
                with self.tm("bab.eval_cand"):
                    sure, amb = self._eval_pairs(cx[cand_rows], cxp[cand_rows], bpart[cand_rows])
                hit = cand_rows[sure | amb]
                if hit.numel():
                    found_idx.append(hit)
            leaf_rows = torch.nonzero(leaf & sel).flatten()
            if leaf_rows.numel():
                # all pairs at the leaf point
                L_ = leaf_rows.numel()
                Pp = pairs.shape[0]
                px = blo[leaf_rows][:, None, :].expand(L_, Pp, n).clone()
                ppx = bplo[leaf_rows][:, None, :].expand(L_, Pp, n).clone()
                px[:, :, self.pa] = values[pairs[:, 0]].to(px.dtype)[None].expand(L_, Pp, -1)
                ppx[:, :, self.pa] = values[pairs[:, 1]].to(px.dtype)[None].expand(L_, Pp, -1)
                lp = bpart[leaf_rows][:, None].expand(L_, Pp)
                sure, amb = self._eval_pairs(px.reshape(-1, n), ppx.reshape(-1, n), lp.reshape(-1))
                flag = (sure | amb).view(L_, Pp)
                anyf = flag.any(dim=1)
                if bool(anyf.any()):
                    first = flag.float().argmax(dim=1)
                    sel_l = torch.nonzero(anyf).flatten()
                    found_idx.append(leaf_rows[sel_l])
                    fx = px[sel_l, first[sel_l]]
                    fxp = ppx[sel_l, first[sel_l]]
                    cx[leaf_rows[sel_l]] = fx
                    cxp[leaf_rows[sel_l]] = fxp
            if found_idx:
                rows = torch.cat(found_idx)
                with self.tm("bab.confirm"):
                    self._confirm(rows, cx, cxp, bpart, status, status_t, cex_x, cex_xp, mlp_exact, exact_models,
                              lo_np, hi_np)
            # ---- split open, non-leaf nodes of running partitions
            nodes_np_now = nodes_t  # device
            budget_ok = nodes_np_now[bpart] < cfg.node_budget
            split = open_ & ~leaf & (status_t[bpart] == RUNNING) & budget_ok
            # partitions that ran out of budget with open nodes -> UNKNOWN
            over = open_ & ~leaf & (status_t[bpart] == RUNNING) & ~budget_ok
            if bool(over.any()):
                status_t[bpart[over]] = UNKNOWN
            sidx = torch.nonzero(split).flatten()
            with self.tm("bab.split"):
                new = self._split(blo[sidx], bhi[sidx], bplo[sidx], bphi[sidx], bpart[sidx], dec.split_dim[sidx])
            # ---- next pool = rest + children
            if self.relaxed:
                clo, chi, cplo, cphi, cpart = new
                xlo = torch.cat([xlo[rest], clo])
                xhi = torch.cat([xhi[rest], chi])
                xplo = torch.cat([xplo[rest], cplo])
                xphi = torch.cat([xphi[rest], cphi])
                part = torch.cat([part[rest], cpart])
            else:
                clo, chi, _, _, cpart = new
                xlo = torch.cat([xlo[rest], clo])
                xhi = torch.cat([xhi[rest], chi])
                xplo, xphi = xlo, xhi
                part = torch.cat([part[rest], cpart])
            if xlo.shape[0] > cfg.max_pool:
                # keep the oldest nodes; partitions losing nodes become UNKNOWN
                lost = torch.unique(part[cfg.max_pool:])
                status_t[lost[status_t[lost] == RUNNING]] = UNKNOWN
                xlo, xhi, part = xlo[:cfg.max_pool], xhi[:cfg.max_pool], part[:cfg.max_pool]
                if self.relaxed:
                    xplo, xphi = xplo[:cfg.max_pool], xphi[:cfg.max_pool]
                else:
                    xplo, xphi = xlo, xhi
        # partitions still running: no nodes left => UNSAT ; nodes left (time budget) => UNKNOWN
        st = status_t.cpu().numpy()
        remaining = set(part.cpu().numpy().tolist()) if xlo.shape[0] else set()
        for p in np.nonzero(st == RUNNING)[0]:
            st[p] = UNKNOWN if p in remaining else UNSAT
        # SAT found on host overrides
        st[status == SAT] = SAT
        nodes_np = nodes_t.cpu().numpy()
        return BaBResult(st.astype(np.int8), cex_x, cex_xp, nodes_np, it, time.time() - t0)

    def _solve_groups(self, groups, lo_np, hi_np, mlp_exact, init_status, exact_models, t0) -> BaBResult:
        """Partitions with different protected-attribute ranges: one solve per PA group (each has
        its own table of PA assignments), results scattered back in input order.  Per-partition
        forced-dead masks and masked exact models follow their partitions into the group."""
        P, n = lo_np.shape
        status = np.full(P, RUNNING, dtype=np.int8) if init_status is None else init_status.astype(np.int8).copy()
        cex_x = np.zeros((P, n), dtype=np.int64)
        cex_xp = np.zeros((P, n), dtype=np.int64)
        nodes = np.zeros(P, dtype=np.int64)
        open_left = np.zeros(P, dtype=np.int64)
        iters = 0
        dead_all = self.dead
        for g in groups:
            sub = BaBSolver(self.be, self.q, replace(self.cfg, time_budget=max(0.0, self.cfg.time_budget -
                                                                                  (time.time() - t0))),
                            dead=None if dead_all is None else dead_all[torch.from_numpy(g).to(dead_all.device)],
                            timer=self.tm)
            em = None if exact_models is None else [exact_models[int(k)] for k in g]
            r = sub.solve(lo_np[g], hi_np[g], mlp_exact, init_status=status[g], exact_models=em)
            status[g], cex_x[g], cex_xp[g], nodes[g] = r.status, r.cex_x, r.cex_xp, r.nodes
            if r.open_left is not None:
                open_left[g] = r.open_left
            iters += r.iters
        return BaBResult(status, cex_x, cex_xp, nodes, iters, time.time() - t0, open_left=open_left)

    # --------------------------------------------------------------------------------------
    def _runtime(self, values_np: np.ndarray, pairs_np: np.ndarray, n_run: int):
        """Native (C++/HIP) BaB runtime checked out of the backend's pool (engine/rtpool.py)."""
        from ..ops import ext
        from ..ops.hip import _net
        from .rtpool import checkout

        rf = refine_level(self.cfg.refine, self.be.widths)
        sm = smear_on(self.cfg.smear, self.be.widths)
        key = (tuple(self.q.pa_idx), tuple(self.q.ra_idx), self.q.tau, values_np.tobytes(), pairs_np.tobytes(),
               bool(self.cfg.crown), int(self.cfg.split_target), rf, sm)
        shared = np.ones(self.q.n, dtype=np.uint8)
        shared[list(self.q.ra_idx)] = 0

        def make(cap):
            return ext().BabRuntime(_net(self.be), self.be.flat.data_ptr(), list(self.q.pa_idx),
                                    values_np.astype(np.float32).reshape(-1).tolist(),
                                    values_np.astype(np.int64).reshape(-1).tolist(),
                                    pairs_np.astype(np.int64).reshape(-1).tolist(),
                                    list(self.q.ra_idx) if self.relaxed else [], float(self.q.tau),
                                    shared.tolist(), int(cap), int(self.cfg.batch_nodes), int(self.cfg.cand_cap),
                                    float(self.be.unit), bool(self.cfg.crown), int(self.cfg.split_target), rf, sm)

        return checkout(self.be, "_bab_rt", key, max(self.cfg.max_pool, n_run), make)

    def _solve_native(self, lo_np, hi_np, status, values_np, pairs_np, mlp_exact, exact_models, t0) -> BaBResult:
        n_run = int((status == RUNNING).sum())
        q = self.q

        def confirm(parts: np.ndarray, buf: np.ndarray) -> np.ndarray:
            with self.tm("bab.confirm"):
                n = q.n
                X = np.rint(buf[:, :n]).astype(np.int64)
                XP = np.rint(buf[:, n:]).astype(np.int64)
                ok = exact.check_pair_constraints(X, XP, lo_np[parts], hi_np[parts], q.pa_idx, q.ra_idx, q.tau)
                out = np.zeros(len(parts), dtype=bool)
                if exact_models is None:
                    idx = np.nonzero(ok)[0]
                    if idx.size:
                        out[idx] = exact.is_violation(mlp_exact, X[idx], XP[idx])
                else:
                    for k in np.nonzero(ok)[0]:
                        out[k] = exact.is_violation(exact_models[int(parts[k])], X[k:k + 1], XP[k:k + 1])[0]
                return out

        dead_ptr = 0
        if self.dead is not None:
            self._dead_u8 = self.dead.to(torch.uint8).contiguous()
            dead_ptr = self._dead_u8.data_ptr()
        stream = torch.cuda.current_stream(self.dev).cuda_stream
        with self.tm("bab.native"), self._runtime(values_np, pairs_np, n_run) as rt:
            rt.set_fuse_settle(bool(self.cfg.fuse_settle))
            st, cx, cxp, nodes, stats = rt.solve(lo_np.astype(np.float32), hi_np.astype(np.float32), status,
                                                  int(self.cfg.node_budget), float(self.cfg.time_budget), dead_ptr,
                                                  confirm, stream, exact_models is None,
                                                  int(self.cfg.escalate_budget), int(self.cfg.escalate_max_w),
                                                  [(int(b), int(o)) for b, o in self.cfg.escalate_steps])
        self.stats = dict(stats)
        with _STATS_LOCK:
            for k in STATS:
                STATS[k] += int(self.stats.get(k, 0))
        return BaBResult(np.asarray(st, dtype=np.int8), np.asarray(cx), np.asarray(cxp), np.asarray(nodes),
                         int(stats["levels"]), time.time() - t0, open_left=np.asarray(stats["open_left"]))

    # --------------------------------------------------------------------------------------
    def _confirm(self, rows, cx, cxp, bpart, status, status_t, cex_x, cex_xp, mlp_exact, exact_models,
                 lo_np, hi_np):
        r = rows.cpu().numpy()
        X = cx[rows].cpu().numpy().round().astype(np.int64)
        XP = cxp[rows].cpu().numpy().round().astype(np.int64)
        parts = bpart[rows].cpu().numpy()
        ok = exact.check_pair_constraints(X, XP, lo_np[parts], hi_np[parts], self.q.pa_idx, self.q.ra_idx,
                                          self.q.tau)
        if exact_models is None:
            viol = exact.is_violation(mlp_exact, X, XP) & ok
        else:
            viol = np.zeros(len(parts), dtype=bool)
            for k, p in enumerate(parts):
                if ok[k]:
                    viol[k] = exact.is_violation(exact_models[p], X[k:k + 1], XP[k:k + 1])[0]
        newly = []
        for k in np.nonzero(viol)[0]:
            p = parts[k]
            if status[p] != SAT:
                status[p] = SAT
                cex_x[p] = X[k]
                cex_xp[p] = XP[k]
                newly.append(p)
        if newly:
            status_t[torch.tensor(newly, device=status_t.device)] = SAT

    def _split(self, lo, hi, plo, phi, part, dim):
        n = lo.shape[1]
        N = lo.shape[0]
        if N == 0:
            e = lo[:0]
            return e, e, e, e, part[:0]
        on_x = dim < n
        d = torch.where(on_x, dim, dim - n)
        ar = torch.arange(N, device=lo.device)
        # children along x dim or x' dim
        src_lo = torch.where(on_x, lo[ar, d], plo[ar, d])
        src_hi = torch.where(on_x, hi[ar, d], phi[ar, d])
        mid = torch.floor((src_lo + src_hi) / 2)
        lo1, hi1, lo2, hi2 = lo.clone(), hi.clone(), lo.clone(), hi.clone()
        plo1, phi1, plo2, phi2 = plo.clone(), phi.clone(), plo.clone(), phi.clone()
        xs = torch.nonzero(on_x).flatten()
        ps = torch.nonzero(~on_x).flatten()
        hi1[xs, d[xs]] = mid[xs]
        lo2[xs, d[xs]] = mid[xs] + 1
        phi1[ps, d[ps]] = mid[ps]
        plo2[ps, d[ps]] = mid[ps] + 1
        clo = torch.cat([lo1, lo2])
        chi = torch.cat([hi1, hi2])
        cplo = torch.cat([plo1, plo2])
        cphi = torch.cat([phi1, phi2])
        cpart = torch.cat([part, part])
        if not self.relaxed:
            return clo, chi, clo, chi, cpart
        # shared dims of x' follow x; tighten the |x_r - x'_r| <= tau coupling
        sh = self.shared
        cplo = torch.where(sh[None, :], clo, cplo)
        cphi = torch.where(sh[None, :], chi, cphi)
        r = self.ra
        t = self.tau
        cplo[:, r] = torch.maximum(cplo[:, r], clo[:, r] - t)
        cphi[:, r] = torch.minimum(cphi[:, r], chi[:, r] + t)
        clo[:, r] = torch.maximum(clo[:, r], cplo[:, r] - t)
        chi[:, r] = torch.minimum(chi[:, r], cphi[:, r] + t)
        ok = torch.all(clo <= chi, dim=1) & torch.all(cplo <= cphi, dim=1)
        return clo[ok], chi[ok], cplo[ok], cphi[ok], cpart[ok]
