"""Neuron pruning stages (sound + heuristic) on batches of partitions.

Reference: ``utils/prune.py`` — ``sound_prune*`` (:671-859), ``dead_node_from_bound``
(:226-251), ``singular_verification*`` (:276-644), ``heuristic_prune`` (:862-939),
``merge_dead_nodes`` (:941-948).  Masks here are boolean tensors ``[P, N]`` over ALL neurons
(hidden layers then the output neuron), matching the reference's per-layer lists; the output
neuron is never pruned by the bound-based stages.

Differences by design (documented in docs/DESIGN.md):
* the per-neuron Z3 check is replaced by the symbolic bound kernel (a neuron whose symbolic
  upper bound is <= 0 on the box is provably dead); the reference's layer-index bug
  (utils/prune.py:271-272 via :304) is not reproduced — the bounds are correct.
* heuristic pruning is reproduced exactly (percentiles with NumPy's linear interpolation) and
  stays flagged as unsound (h_attempt / h_success columns).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch


def layer_slices(widths: Sequence[int]) -> List[slice]:
    out, off = [], 0
    for w in widths:
        out.append(slice(off, off + w))
        off += w
    return out


def ensure_one_alive(dead: torch.Tensor, widths: Sequence[int]) -> torch.Tensor:
    """``if not 0 in l: l[0] = 0`` per layer (utils/prune.py:689-691)."""
    dead = dead.clone()
    for sl in layer_slices(widths):
        all_dead = dead[:, sl].all(dim=1)
        if bool(all_dead.any()):
            dead[all_dead, sl.start] = False
    return dead


def candidates_from_counts(counts: torch.Tensor, n_samples: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """``candidate_dead_nodes`` (utils/prune.py:168-192): never-active neurons + pos_prob."""
    cand = counts == 0
    pos_prob = counts.to(torch.float32) / float(n_samples)
    return cand, pos_prob


def bound_dead(cand: torch.Tensor, ub_hidden: torch.Tensor, widths: Sequence[int]) -> Tuple[torch.Tensor, torch.Tensor]:
    """``dead_node_from_bound``: a candidate hidden neuron with upper bound <= 0 is dead.

    ``ub_hidden`` [P, N_hidden]; returns (dead [P, N], remaining candidates [P, N]).  For the
    output layer the reference keeps the candidate flag as the mask (:233-240); reproduced.
    """
    Nh = ub_hidden.shape[1]
    dead = cand.clone()
    hid = cand[:, :Nh] & (ub_hidden <= 0)
    dead[:, :Nh] = hid
    rem = cand.clone()
    rem[:, :Nh] = cand[:, :Nh] & ~hid
    return dead, rem


def merge(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return a | b


def compression(dead: torch.Tensor) -> torch.Tensor:
    """Per-partition compression ratio (utils/prune.py:194-203), output layer included."""
    return dead.to(torch.float32).mean(dim=1)


def _masked_percentile(vals: torch.Tensor, mask: torch.Tensor, q: float):
    """Row-wise NumPy-'linear' percentile of ``vals`` over entries where ``mask`` (>=1 entry)."""
    inf = torch.full_like(vals, float("inf"))
    srt = torch.sort(torch.where(mask, vals, inf), dim=1).values
    k = mask.sum(dim=1).clamp(min=1)
    pos = (k - 1).to(vals.dtype) * (q / 100.0)
    lo = pos.floor().long()
    hi = torch.minimum(lo + 1, k - 1)
    frac = pos - lo.to(vals.dtype)
    a = srt.gather(1, lo[:, None])[:, 0]
    b = srt.gather(1, hi[:, None])[:, 0]
    return a + (b - a) * frac


def heuristic_prune_batch(ws_lb: torch.Tensor, ws_ub: torch.Tensor, cand: torch.Tensor, s_cand: torch.Tensor,
                          deads: torch.Tensor, widths: Sequence[int], perc: float):
    """Vectorised :func:`heuristic_prune_one` over a batch of partitions (rows).

    Same decisions as the reference ``heuristic_prune`` (utils/prune.py:862-939): per hidden
    layer compare the candidates' and non-candidates' ``ws_ub`` distributions (mean, median,
    NumPy-linear percentiles) and mark harsh outliers dead.  Returns (new, merged) [P, N] bool.
    """
    dt = torch.float64
    lb = ws_lb.to(dt)
    ub = ws_ub.to(dt)
    new = torch.zeros_like(cand, dtype=torch.bool)
    sls = layer_slices(widths)
    for sl in sls[:-1]:
        c = cand[:, sl].bool()
        u = ub[:, sl]
        l = lb[:, sl]
        nc = ~c
        kc = c.sum(1)
        kn = nc.sum(1)
        zero = torch.zeros_like(u)
        mean_c = torch.where(c, u, zero).sum(1) / kc.clamp(min=1)
        mean_n = torch.where(nc, u, zero).sum(1) / kn.clamp(min=1)
        med_c = _masked_percentile(u, c, 50.0)
        med_n = _masked_percentile(u, nc, 50.0)
        p5 = _masked_percentile(u, nc, perc)
        p95 = _masked_percentile(u, nc, 100.0 - perc)
        differ = (mean_n > 2 * mean_c) & (med_n > 2 * med_c) & (kn > 0) & (kc > 0)
        hit = s_cand[:, sl].bool() & (u < p5[:, None]) & (u < 0.1 * p95[:, None]) & (u < l.abs())
        layer_new = torch.where(differ[:, None], hit, torch.zeros_like(hit))
        layer_new = layer_new | (kn == 0)[:, None]
        new[:, sl] = layer_new
    for sl in sls:
        alld = new[:, sl].all(1)
        new[alld, sl.start] = False
    merged = deads.bool() | new
    for sl in sls:
        alld = merged[:, sl].all(1)
        merged[alld, sl.start] = False
    return new, merged


def heuristic_prune_one(ws_lb: np.ndarray, ws_ub: np.ndarray, cand: np.ndarray, s_cand: np.ndarray,
                        deads: np.ndarray, widths: Sequence[int], perc: float) -> Tuple[np.ndarray, np.ndarray]:
    """Reference ``heuristic_prune`` for ONE partition; arrays over all N neurons.

    Returns (new heuristic deads, merged deads), both [N] bool.
    """
    new = np.zeros_like(cand, dtype=bool)
    sls = layer_slices(widths)
    for li, sl in enumerate(sls[:-1]):
        c = cand[sl].astype(bool)
        ub = ws_ub[sl]
        lb = ws_lb[sl]
        cv, nv = ub[c], ub[~c]
        if nv.size == 0:
            new[sl] = True
        elif cv.size == 0:
            pass
        else:
            if nv.mean() > 2 * cv.mean() and np.median(nv) > 2 * np.median(cv):
                p5 = np.percentile(nv, perc)
                p95 = np.percentile(nv, 100 - perc)
                sc = s_cand[sl].astype(bool)
                hit = sc & (ub < p5) & (ub < 0.1 * p95) & (ub < np.abs(lb))
                new[sl] = hit
    for sl in sls:
        if new[sl].all():
            new[sl.start] = False
    merged = deads.astype(bool) | new
    for sl in sls:
        if merged[sl].all():
            merged[sl.start] = False
    return new, merged
