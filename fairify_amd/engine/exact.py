"""Exact sign of the network logit at integer points (counterexample confirmation).

The reference's Z3 encoding evaluates the network in exact rational arithmetic over the fp32
weight values (``z3_net`` uses ``ToReal``; utils/AC-1-Model-Functions.py:36-39), and its
counterexamples are replayed with ``net`` (src/AC/Verify-AC.py:229-254).  Here a candidate
pair found on the GPU is confirmed by an fp64 forward with a rigorous rounding bound; only
rows whose logit is within that bound of 0 fall back to exact ``fractions.Fraction``
arithmetic, so every reported SAT is a true violation of the exact network.
"""
from __future__ import annotations

from fractions import Fraction
from typing import List, Sequence

import numpy as np

from ..models.mlp import MLP

U64 = 2.0 ** -53


def _gamma(k: int) -> float:
    ku = (k + 2) * U64
    return ku / (1 - ku)


def logits_with_error(mlp: MLP, X: np.ndarray, with_magnitude: bool = False):
    """fp64 logits, their rigorous rounding bound, and (``with_magnitude``) the magnitude bound
    m = |W|^T m + |b| of the logit (m == 0 exactly <=> every term feeding it is exactly 0)."""
    h = np.asarray(X, dtype=np.float64)
    m = np.abs(h)
    e = np.zeros_like(h)
    for l, (w, b) in enumerate(zip(mlp.weights, mlp.biases)):
        w64 = w.astype(np.float64)
        b64 = b.astype(np.float64)
        g = _gamma(w.shape[0] + 1)
        aw = np.abs(w64)
        z = h @ w64 + b64
        e = (e + g * m) @ aw + g * np.abs(b64)
        m = m @ aw + np.abs(b64)
        if l < mlp.n_layers - 1:
            h = np.maximum(z, 0)
            # certainly negative pre-activation (z + e < 0): the exact ReLU output is exactly 0,
            # so that neuron carries no value, magnitude or error into the next layer
            dead = z + e < 0
            h[dead] = 0.0
            m = np.where(dead, 0.0, m)
            e = np.where(dead, 0.0, e)
        else:
            h = z
    if with_magnitude:
        return h[:, 0], e[:, 0] * 1.0001 + 1e-300, m[:, 0]
    return h[:, 0], e[:, 0] * 1.0001 + 1e-300


def exact_logit_fraction(mlp: MLP, x: Sequence[int]) -> Fraction:
    h: List[Fraction] = [Fraction(int(v)) for v in x]
    for l, (w, b) in enumerate(zip(mlp.weights, mlp.biases)):
        W = [[Fraction(float(w[i, j])) for j in range(w.shape[1])] for i in range(w.shape[0])]
        nxt = []
        for j in range(w.shape[1]):
            s = Fraction(float(b[j]))
            for i in range(w.shape[0]):
                if h[i] != 0 and W[i][j] != 0:
                    s += h[i] * W[i][j]
            if l < mlp.n_layers - 1 and s < 0:
                s = Fraction(0)
            nxt.append(s)
        h = nxt
    return h[0]


def exact_signs(mlp: MLP, X: np.ndarray) -> np.ndarray:
    """Exact sign (-1, 0, +1) of the logit for integer rows ``X`` [B, n0]."""
    X = np.asarray(X)
    if X.shape[0] == 0:
        return np.zeros(0, dtype=np.int64)
    z, e, m = logits_with_error(mlp, X, with_magnitude=True)
    s = np.sign(z).astype(np.int64)
    # m == 0: products of fp32 weights and integers are exact in fp64 and sums of non-negative
    # terms round to 0 only when every term is 0, so the exact logit is 0 (no Fraction needed)
    s[m == 0.0] = 0
    amb = (np.abs(z) <= e) & (m != 0.0)
    for i in np.nonzero(amb)[0]:
        v = exact_logit_fraction(mlp, X[i])
        s[i] = (v > 0) - (v < 0)
    return s


def is_violation(mlp: MLP, x: np.ndarray, xp: np.ndarray) -> np.ndarray:
    """Exact test of the fairness post-condition for row pairs (strict opposite signs)."""
    sx = exact_signs(mlp, x)
    sxp = exact_signs(mlp, xp)
    return (sx * sxp) < 0


def check_pair_constraints(x: np.ndarray, xp: np.ndarray, lo: np.ndarray, hi: np.ndarray,
                           pa_idx, ra_idx, tau: int) -> np.ndarray:
    """Pre-condition of the query for pairs (x, x') against their partition boxes."""
    x = np.asarray(x, dtype=np.int64)
    xp = np.asarray(xp, dtype=np.int64)
    ok = np.all((x >= lo) & (x <= hi), axis=1)
    n = x.shape[1]
    pa = list(pa_idx)
    ra = list(ra_idx)
    free = [i for i in range(n) if i not in pa and i not in ra]
    if pa:
        ok &= np.all(x[:, pa] != xp[:, pa], axis=1)
        ok &= np.all((xp[:, pa] >= lo[:, pa]) & (xp[:, pa] <= hi[:, pa]), axis=1)
    if free:
        ok &= np.all(x[:, free] == xp[:, free], axis=1)
    if ra:
        ok &= np.all(np.abs(x[:, ra] - xp[:, ra]) <= tau, axis=1)
    return ok
