"""Simulation stage: random lattice points per partition (K3) + falsification (K8).

Reference: ``simluate_data`` (utils/prune.py:205-222) draws ``sim_size`` uniform integer points
per box with ``np.random.randint``; ``candidate_dead_nodes`` (:168-192) forwards each point
through ``layer_net`` to find never-active neurons.  Here the points come from a counter-based
hash (reproducible, identical on host and device), the activation counts are produced in one
batched pass, and the same points double as a falsifier: every point is re-evaluated with all
other protected-attribute values (and random relaxed offsets) and any strict sign flip becomes
a SAT candidate, later confirmed exactly.  A short bisection between points of opposite sign
(boundary walk) adds candidates close to the decision boundary.

On the GPU the whole profile+falsify pass is one fused HIP kernel (``fa_sim_kernel``: points
never touch HBM); the boundary walk reuses the HIP forward kernel.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from ..ops import reference as ref
from ..ops.backend import Backend
from ..spec import ResolvedQuery


@dataclass
class SimResult:
    counts: torch.Tensor          # [P, N] activation counts (all neurons)
    found: torch.Tensor           # [P] bool  candidate violation found
    wit_x: torch.Tensor           # [P, n0]
    wit_xp: torch.Tensor          # [P, n0]


def _flips(z: torch.Tensor, zp: torch.Tensor, pairs: torch.Tensor) -> torch.Tensor:
    zi = z[..., pairs[:, 0]]
    zj = zp[..., pairs[:, 1]]
    return ((zi < 0) & (zj > 0)) | ((zi > 0) & (zj < 0))


def boundary_walk(be: Backend, q: ResolvedQuery, lo, hi, pids, n_samples: int, seed: int, values, pairs,
                  res: SimResult, z0: torch.Tensor, k: int, steps: int) -> None:
    """Bisect between the k most positive and k most negative samples (logit at PA value 0),
    on lattice points, checking every PA pair at each probe; fills ``res`` for partitions
    without a witness yet."""
    P, n = lo.shape
    dev = lo.device
    nf = ~res.found
    if not bool(nf.any()) or n_samples == 0:
        return
    sel = torch.nonzero(nf).flatten()
    lo_s, hi_s, pid_s, z0s = lo[sel], hi[sel], pids[sel], z0[sel]
    k = min(k, n_samples)
    top = z0s.topk(k, dim=1).indices
    bot = (-z0s).topk(k, dim=1).indices
    A = ref.sample_points_at(lo_s, hi_s, pid_s, top, seed)
    Bp = ref.sample_points_at(lo_s, hi_s, pid_s, bot, seed)
    ar = torch.arange(sel.numel(), device=dev)[:, None]
    ok = (z0s[ar, top] > 0) & (z0s[ar, bot] < 0)
    pa = torch.tensor(list(q.pa_idx), device=dev, dtype=torch.long)
    vals = values.to(torch.float32)
    V = vals.shape[0]
    p_ = sel.numel()
    tlo = torch.zeros(p_, k, device=dev)
    thi = torch.ones(p_, k, device=dev)
    done = torch.zeros(p_, dtype=torch.bool, device=dev)
    for _ in range(steps):
        tm = 0.5 * (tlo + thi)
        M = torch.round(A + tm[..., None] * (Bp - A))
        MV = M[:, :, None, :].expand(p_, k, V, n).clone()
        MV[:, :, :, pa] = vals[None, None].expand(p_, k, V, -1)
        zm = be.forward(MV.reshape(-1, n)).view(p_, k, V)
        fl = _flips(zm, zm, pairs) & ok[..., None]
        hit = fl.flatten(1).any(dim=1) & ~done
        if bool(hit.any()):
            idx = fl.flatten(1).float().argmax(dim=1)
            kk = idx // pairs.shape[0]
            pi = idx % pairs.shape[0]
            a1 = torch.arange(p_, device=dev)
            g = torch.nonzero(hit).flatten()
            tgt = sel[g]
            res.found[tgt] = True
            res.wit_x[tgt] = MV[a1, kk, pairs[pi, 0]][g]
            res.wit_xp[tgt] = MV[a1, kk, pairs[pi, 1]][g]
            done |= hit
        pos = zm[:, :, 0] > 0
        tlo = torch.where(pos, tm, tlo)
        thi = torch.where(pos, thi, tm)


def simulate(be: Backend, q: ResolvedQuery, lo: torch.Tensor, hi: torch.Tensor, pids: torch.Tensor,
             n_samples: int, seed: int, values: torch.Tensor, pairs: torch.Tensor,
             bisect_pairs: int = 16, bisect_steps: int = 12, sub: int = 256) -> SimResult:
    """Profile + falsify ``P`` partitions. ``values`` [V, k] PA assignments, ``pairs`` [Pp, 2]."""
    if be.hip:
        from ..ops import hip

        return hip.simulate(be, q, lo, hi, pids, n_samples, seed, values, pairs, bisect_pairs, bisect_steps)
    P, n = lo.shape
    dev = lo.device
    pa = torch.tensor(list(q.pa_idx), device=dev, dtype=torch.long)
    ra = torch.tensor(list(q.ra_idx), device=dev, dtype=torch.long)
    V = values.shape[0]
    Pp = pairs.shape[0]
    counts = torch.zeros(P, be.mlp.n_neurons, dtype=torch.int32, device=dev)
    res = SimResult(counts=counts, found=torch.zeros(P, dtype=torch.bool, device=dev),
                    wit_x=torch.zeros(P, n, device=dev), wit_xp=torch.zeros(P, n, device=dev))
    z0 = torch.zeros(P, n_samples, device=dev)
    vals = values.to(torch.float32)
    for s0 in range(0, P, sub):
        sl = slice(s0, min(P, s0 + sub))
        X = ref.sample_points(lo[sl], hi[sl], pids[sl], n_samples, seed)          # [p, S, n]
        counts[sl] = be.activation_counts(X)
        p_, S = X.shape[0], X.shape[1]
        XV = X[:, :, None, :].expand(p_, S, V, n).clone()
        XV[:, :, :, pa] = vals[None, None].expand(p_, S, V, -1)
        XPV = XV
        if q.relaxed:
            h = ref.rng_u32(seed ^ 0x2545F491, pids[sl].to(torch.int64)[:, None, None],
                            torch.arange(S, device=dev)[None, :, None], ra[None, None, :])
            off = (h % (2 * q.tau + 1)).to(torch.float32) - q.tau
            XPV = XV.clone()
            XPV[:, :, :, ra] = XV[:, :, :, ra] + off[:, :, None, :]
        z = be.forward(XV.reshape(-1, n)).view(p_, S, V)
        zp = z if not q.relaxed else be.forward(XPV.reshape(-1, n)).view(p_, S, V)
        z0[sl] = z[:, :, 0]
        flip = _flips(z, zp, pairs)                                                # [p, S, Pp]
        anyf = flip.flatten(1).any(dim=1)
        if bool(anyf.any()):
            idx = flip.flatten(1).float().argmax(dim=1)
            si, pi = idx // Pp, idx % Pp
            ar = torch.arange(p_, device=dev)
            g = torch.nonzero(anyf).flatten()
            res.found[sl][g] = True
            res.wit_x[sl][g] = XV[ar, si, pairs[pi, 0]][g]
            res.wit_xp[sl][g] = XPV[ar, si, pairs[pi, 1]][g]
    if bisect_pairs and bisect_steps:
        boundary_walk(be, q, lo, hi, pids, n_samples, seed, values, pairs, res, z0, bisect_pairs, bisect_steps)
    return res
