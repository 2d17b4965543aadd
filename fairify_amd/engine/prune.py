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
