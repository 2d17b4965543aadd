"""Themis-style causal-discrimination testing (C29), batched on the device (K11).

Reference: ``CausalDiscriminationDetector`` (src/AC/metrics.py:40-288): draw random assignments
of the non-protected features from each feature's observed values, flip the protected
features through every other assignment, count samples whose prediction changes; stop once
the normal-approximation confidence half-width drops below ``margin`` (after ``min_samples``),
at most ``max_samples``.  The reference issues one single-row Keras ``predict`` per candidate
(~2 000 calls); here all ``max_samples x |PA assignments|`` rows are generated at once and
classified by ONE batched forward, and the sequential stopping rule is evaluated on the
cumulative counts (same decision sequence for the same sample stream).
"""
from __future__ import annotations

import itertools
import math
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np


def _z(conf: float) -> float:
    from scipy.stats import norm

    return float(norm.ppf(conf))


class CausalDiscriminationDetector:
    def __init__(self, predict: Callable[[np.ndarray], np.ndarray], feature_names: Sequence[str],
                 max_samples: int = 1000, min_samples: int = 100, seed: int = 42):
        """``predict`` maps rows [B, n] -> labels [B] (batched; e.g. a Backend forward > 0)."""
        self.predict = predict
        self.names = list(feature_names)
        self.values: Dict[str, np.ndarray] = {}
        self.max_samples = max_samples
        self.min_samples = min_samples
        self.rng = np.random.default_rng(seed)

    def add_feature(self, name: str, values) -> None:
        self.values[name] = np.asarray(sorted(set(np.asarray(values).tolist())), dtype=np.float64)

    def add_continuous_feature(self, name: str, lo: float, hi: float, num_values: int = 10) -> None:
        self.values[name] = np.linspace(lo, hi, num_values)

    @classmethod
    def from_data(cls, predict, X: np.ndarray, names: Sequence[str], **kw) -> "CausalDiscriminationDetector":
        d = cls(predict, names, **kw)
        for i, n in enumerate(names):
            d.add_feature(n, np.unique(X[:, i]))
        return d

    def causal_discrimination(self, protected: Sequence[str], conf: float = 0.999, margin: float = 0.0001
                              ) -> Tuple[int, float, List[Tuple[np.ndarray, np.ndarray]]]:
        """Returns (samples used, discrimination rate, discriminating pairs)."""
        assert protected, "must specify protected features"
        S = self.max_samples - 1               # reference: range(1, max_samples)
        n = len(self.names)
        pidx = [self.names.index(p) for p in protected]
        base = np.zeros((S, n))
        for i, name in enumerate(self.names):
            vals = self.values[name]
            base[:, i] = vals[self.rng.integers(0, len(vals), size=S)]
        combos = np.array(list(itertools.product(*[self.values[p] for p in protected])))   # [C, k]
        C = combos.shape[0]
        rows = np.repeat(base[:, None, :], C, axis=1)
        rows[:, :, pidx] = combos[None]
        preds = np.asarray(self.predict(rows.reshape(S * C, n))).reshape(S, C)
        orig = preds[np.arange(S), np.argmax(np.all(combos[None] == base[:, None, pidx], axis=2), axis=1)]
        flip = (preds != orig[:, None]).any(axis=1)
        counts = np.cumsum(flip)
        k = np.arange(1, S + 1)
        rate = counts / k
        err = np.where((rate == 0) | (rate == 1), 0.0, _z(conf) * np.sqrt(rate * (1 - rate) / k))
        stop = (k >= self.min_samples) & (err < margin)
        used = int(np.argmax(stop)) + 1 if stop.any() else S
        pairs = []
        for s in np.nonzero(flip[:used])[0]:
            c = int(np.argmax(preds[s] != orig[s]))
            alt = base[s].copy()
            alt[pidx] = combos[c]
            pairs.append((base[s].copy(), alt))
        return used, float(counts[used - 1] / used) if used >= self.min_samples else 0.0, pairs

    def discrimination_search(self, threshold: float = 0.15, conf: float = 0.99, margin: float = 0.01):
        found: Dict[Tuple[str, ...], Dict] = {}
        for size in range(1, len(self.names)):
            for combo in itertools.combinations(self.names, size):
                if any(set(k).issubset(combo) for k in found):
                    continue
                _, rate, pairs = self.causal_discrimination(list(combo), conf, margin)
                if rate > threshold:
                    found[combo] = {"rate": rate, "pairs": pairs}
        return found
