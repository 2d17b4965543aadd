"""``analyze`` command: group metrics, causal discrimination and hybrid routing of a model.

Mirrors the tail of the fork's experiment driver (src/AC/Verify-AC-experiment-new2.py:562-781):
original vs fairer vs hybrid accuracy, CNT consistency and causal-discrimination rates, plus
the per-model AIF360-style metric row (src/AC/Verify-AC-experiment-new.py:482-542).
"""
from __future__ import annotations

import json
import os
from typing import Dict, Optional

import numpy as np
import torch

from .. import presets
from ..data import tabular
from ..models.zoo import get_model
from ..ops.backend import Backend
from .causal import CausalDiscriminationDetector
from .hybrid import VerdictTable, hybrid_predict
from .metrics import all_metrics


def _predictor(mlp, device):
    be = Backend(mlp, device=device)

    def predict(X: np.ndarray) -> np.ndarray:
        out = []
        for s in range(0, len(X), 1 << 18):
            x = torch.as_tensor(np.asarray(X[s:s + (1 << 18)], dtype=np.float32), device=be.device)
            out.append((be.forward(x) > 0).to(torch.int64).cpu().numpy())
        return np.concatenate(out) if out else np.zeros(0, dtype=np.int64)

    return predict


def analyze_model(preset: str, model: str, fairer: Optional[str] = None, results: Optional[str] = None,
                  weights: str = "zoo", seed: int = 0, out_dir: Optional[str] = None, device: str = "cpu",
                  causal_samples: int = 1000) -> Dict:
    pre = presets.get(preset)
    dom = pre.domain()
    q = pre.resolved()
    pa = q.pa_idx[0]
    mlp = get_model(model, weights=weights, seed=seed)
    ds = tabular.load(pre.suite, seed=seed, mlp=mlp)
    X, y = ds.X_test, ds.y_test
    p_orig = _predictor(mlp, device)
    res: Dict = {"model": model, "preset": preset, "data": "synthetic" if ds.synthetic else ds.name,
                 "n_test": int(len(y))}
    res["original"] = all_metrics(X, y, p_orig(X), pa, device=device)
    names = ds.columns
    pa_names = [names[i] for i in q.pa_idx]
    cd = CausalDiscriminationDetector.from_data(p_orig, np.concatenate([ds.X_train, X]), names,
                                                max_samples=causal_samples, seed=seed)
    res["original"]["causal"] = cd.causal_discrimination(pa_names)[1]
    if fairer:
        fm = get_model(fairer, weights=weights, seed=seed) if not os.path.exists(fairer) else _load(fairer)
        p_fair = _predictor(fm, device)
        res["fairer"] = all_metrics(X, y, p_fair(X), pa, device=device)
        cd.predict = p_fair
        cd.rng = np.random.default_rng(seed)
        res["fairer"]["causal"] = cd.causal_discrimination(pa_names)[1]
        if results:
            grid = pre.grid(seed=seed)
            table = VerdictTable.from_csv(grid, os.path.join(results, f"{model}.csv"), seed=seed)
            yh = hybrid_predict(X, table, p_orig, p_fair)
            res["hybrid"] = all_metrics(X, y, yh, pa, device=device)
            res["verdicts"] = table.counts()

            def p_h(Z):
                return hybrid_predict(Z, table, p_orig, p_fair)

            cd.predict = p_h
            cd.rng = np.random.default_rng(seed)
            res["hybrid"]["causal"] = cd.causal_discrimination(pa_names)[1]
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, f"{model}-analysis.json"), "w") as f:
            json.dump(res, f, indent=2, default=float)
    return res


def _load(path: str):
    from ..models.mlp import MLP

    if path.endswith(".h5"):
        from ..models.keras_io import load_keras_h5

        return load_keras_h5(path)
    return MLP.load_npz(path)
