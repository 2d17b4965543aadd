"""ReLU MLP container used by every stage of the verifier.

Replaces the 53 hand-unrolled per-model encodings of the reference
(``utils/*-Model-Functions.py``: ``layer_net``/``net``/``z3_net``, e.g.
``utils/AC-1-Model-Functions.py:16-48``) with one generic container: weights in Keras
layout ``W_l [n_{l-1}, n_l]`` fp32, biases ``b_l [n_l]``, ReLU on every hidden layer, linear
last layer (the pre-sigmoid logit the fairness property is stated on).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np


@dataclass
class MLP:
    weights: List[np.ndarray]
    biases: List[np.ndarray]
    name: str = "mlp"

    def __post_init__(self):
        self.weights = [np.ascontiguousarray(w, dtype=np.float32) for w in self.weights]
        self.biases = [np.ascontiguousarray(b, dtype=np.float32).reshape(-1) for b in self.biases]
        assert len(self.weights) == len(self.biases) and len(self.weights) >= 1
        for l, (w, b) in enumerate(zip(self.weights, self.biases)):
            assert w.ndim == 2 and w.shape[1] == b.shape[0], (l, w.shape, b.shape)
            if l:
                assert w.shape[0] == self.weights[l - 1].shape[1]
        assert self.weights[-1].shape[1] == 1, "binary classifier with one logit expected"

    # ---------------------------------------------------------------- shape helpers
    @property
    def n_in(self) -> int:
        return int(self.weights[0].shape[0])

    @property
    def widths(self) -> List[int]:
        """Output width of every layer (hidden layers then the logit)."""
        return [int(w.shape[1]) for w in self.weights]

    @property
    def hidden(self) -> List[int]:
        return self.widths[:-1]

    @property
    def n_layers(self) -> int:
        return len(self.weights)

    @property
    def n_neurons(self) -> int:
        return int(sum(self.widths))

    def describe(self) -> str:
        return f"{self.name}: {self.n_in}->" + "-".join(str(h) for h in self.hidden) + "->1"

    # ---------------------------------------------------------------- evaluation (host, fp64)
    def layer_outputs(self, x: np.ndarray, dtype=np.float64) -> List[np.ndarray]:
        """Post-activation output of every layer (last layer linear) — ``layer_net``."""
        h = np.asarray(x, dtype=dtype)
        outs = []
        for l, (w, b) in enumerate(zip(self.weights, self.biases)):
            h = h @ w.astype(dtype) + b.astype(dtype)
            if l < self.n_layers - 1:
                h = np.maximum(h, 0)
            outs.append(h)
        return outs

    def logits(self, x: np.ndarray, dtype=np.float64) -> np.ndarray:
        """Pre-sigmoid logit(s) — ``net``."""
        return self.layer_outputs(x, dtype)[-1][..., 0]

    def predict(self, x: np.ndarray) -> np.ndarray:
        """Class labels (sigmoid > 0.5  <=>  logit > 0) — ``get_y_pred``."""
        return (self.logits(x) > 0).astype(np.int64)

    def proba(self, x: np.ndarray) -> np.ndarray:
        z = self.logits(x)
        return 0.5 * (1.0 + np.tanh(0.5 * z))

    # ---------------------------------------------------------------- surgery
    def prune(self, dead: Sequence[np.ndarray]) -> "MLP":
        """Delete dead neurons (``prune_neurons``, utils/prune.py:950-977).

        ``dead[l][j]`` true => neuron j of layer l removed (column of W_l, entry of b_l, row of
        W_{l+1}).  The output neuron is never removed.
        """
        ws = [w.copy() for w in self.weights]
        bs = [b.copy() for b in self.biases]
        for l in range(self.n_layers - 1):
            keep = ~np.asarray(dead[l], dtype=bool)
            if not keep.any():
                keep[0] = True
            ws[l] = ws[l][:, keep]
            bs[l] = bs[l][keep]
            ws[l + 1] = ws[l + 1][keep, :]
        return MLP(ws, bs, name=self.name)

    def masked(self, dead: Sequence[np.ndarray]) -> "MLP":
        """Same function as :meth:`prune` but keeps shapes (dead neurons' outgoing weights zeroed)."""
        ws = [w.copy() for w in self.weights]
        bs = [b.copy() for b in self.biases]
        for l in range(self.n_layers - 1):
            d = np.asarray(dead[l], dtype=bool)
            ws[l][:, d] = 0
            bs[l][d] = 0
        return MLP(ws, bs, name=self.name)

    def flat_params(self) -> np.ndarray:
        return np.concatenate([np.concatenate([w.reshape(-1), b]) for w, b in zip(self.weights, self.biases)])

    # ---------------------------------------------------------------- torch interop
    def to_torch(self, device="cpu"):
        import torch

        mods = []
        for l, (w, b) in enumerate(zip(self.weights, self.biases)):
            lin = torch.nn.Linear(w.shape[0], w.shape[1])
            with torch.no_grad():
                lin.weight.copy_(torch.from_numpy(w.T.copy()))
                lin.bias.copy_(torch.from_numpy(b))
            mods.append(lin)
            if l < self.n_layers - 1:
                mods.append(torch.nn.ReLU())
        return torch.nn.Sequential(*mods).to(device)

    @classmethod
    def from_torch(cls, seq, name: str = "mlp") -> "MLP":
        import torch

        ws, bs = [], []
        for m in seq:
            if isinstance(m, torch.nn.Linear):
                ws.append(m.weight.detach().cpu().numpy().T.copy())
                bs.append(m.bias.detach().cpu().numpy().copy())
        return cls(ws, bs, name=name)

    # ---------------------------------------------------------------- persistence (.npz, no pickle)
    def save_npz(self, path: str) -> None:
        arrs = {}
        for l, (w, b) in enumerate(zip(self.weights, self.biases)):
            arrs[f"W{l}"] = w
            arrs[f"b{l}"] = b
        np.savez(path, name=np.array(self.name), **arrs)

    @classmethod
    def load_npz(cls, path: str) -> "MLP":
        z = np.load(path, allow_pickle=False)
        L = sum(1 for k in z.files if k.startswith("W"))
        name = str(z["name"]) if "name" in z.files else "mlp"
        return cls([z[f"W{l}"] for l in range(L)], [z[f"b{l}"] for l in range(L)], name=name)


def compression_ratio(dead: Sequence[np.ndarray]) -> float:
    """Fraction of removed neurons over ALL layers incl. the output (utils/prune.py:194-203)."""
    tot = sum(int(np.asarray(d).size) for d in dead)
    if tot == 0:
        return 0.0
    return float(sum(int(np.asarray(d, dtype=bool).sum()) for d in dead)) / tot


def random_mlp(n_in: int, hidden: Sequence[int], seed: int = 0, name: str = "mlp",
               init: str = "glorot_uniform", bias_scale: float = 0.0) -> MLP:
    """Random-init MLP (Keras default glorot_uniform kernels, zero biases)."""
    rng = np.random.default_rng(seed)
    dims = [n_in] + list(hidden) + [1]
    ws, bs = [], []
    for a, b in zip(dims[:-1], dims[1:]):
        if init == "glorot_uniform":
            lim = np.sqrt(6.0 / (a + b))
            w = rng.uniform(-lim, lim, size=(a, b))
        elif init == "he_normal":
            w = rng.normal(0, np.sqrt(2.0 / a), size=(a, b))
        else:
            raise ValueError(init)
        ws.append(w.astype(np.float32))
        bs.append((rng.uniform(-bias_scale, bias_scale, size=b) if bias_scale else np.zeros(b)).astype(np.float32))
    return MLP(ws, bs, name=name)
