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
from .hybrid import VerdictTable, case_breakdown, hybrid_predict
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
            res["cases"] = case_breakdown(X, table)

            def p_h(Z):
                return hybrid_predict(Z, table, p_orig, p_fair)

            cd.predict = p_h
            cd.rng = np.random.default_rng(seed)
            res["hybrid"]["causal"] = cd.causal_discrimination(pa_names)[1]
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, f"{model}-analysis.json"), "w") as f:
            json.dump(res, f, indent=2, default=float)
        if "hybrid" in res:
            write_hybrid_csvs(res, model, fairer, out_dir, n_test=len(y))
    return res


_MCOLS = ("accuracy", "DI", "SPD", "EOD", "AOD", "ERD", "CNT", "TI")


def write_hybrid_csvs(res: Dict, model: str, fairer: str, out_dir: str, n_test: int) -> None:
    """``hybrid_approach_results.csv`` and ``debug_case_breakdown.csv`` in the fork's layout
    (src/AC/Verify-AC-experiment-new.py:760-816)."""
    import csv

    fname = os.path.splitext(os.path.basename(fairer))[0]
    with open(os.path.join(out_dir, "hybrid_approach_results.csv"), "w", newline="") as fp:
        wr = csv.writer(fp, dialect="excel")
        wr.writerow(["Approach", "Accuracy", "DI", "SPD", "EOD", "AOD", "ERD", "CNT", "TI"])
        for label, key in (("Hybrid", "hybrid"), (f"{model} Original", "original"), (f"{fname} Fairer", "fairer")):
            wr.writerow([label] + [res[key][c] for c in _MCOLS])
    c = res["cases"]
    orig_used = c["no_partition"] + c["unsat_original"] + c["unknown_original"]
    pct = lambda k: f"{k / max(1, n_test) * 100:.2f}%"
    rows = [
        ["Case", "Description", "Model Used", "Count", "Percentage"],
        ["Case 1", "No partition found", model, c["no_partition"], pct(c["no_partition"])],
        ["Case 3", "SAT/Unfair partition", fname, c["sat_fairer"], pct(c["sat_fairer"])],
        ["Case 4", "UNSAT/Fair partition", model, c["unsat_original"], pct(c["unsat_original"])],
        ["Case 5", "Unknown partition", model, c["unknown_original"], pct(c["unknown_original"])],
        ["", "", "", "", ""],
        ["SUMMARY", f"Total {model} used", model, orig_used, pct(orig_used)],
        ["SUMMARY", f"Total {fname} used", fname, c["sat_fairer"], pct(c["sat_fairer"])],
    ]
    with open(os.path.join(out_dir, "debug_case_breakdown.csv"), "w", newline="") as fp:
        csv.writer(fp, dialect="excel").writerows(rows)


def _load(path: str):
    from ..models.mlp import MLP

    if path.endswith(".h5"):
        from ..models.keras_io import load_keras_h5

        return load_keras_h5(path)
    return MLP.load_npz(path)
