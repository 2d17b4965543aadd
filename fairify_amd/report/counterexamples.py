"""Counterexample export with label decoding (C26).

Reference: ``decode_counterexample`` + ``counterexample.csv`` writers of the fork
(src/AC/Verify-AC-experiment-new2.py:344-407, src/GC/...-new2.py:318-467,
src/BM/...-new2.py:343-404): encoded integers are mapped back to category strings with the
training LabelEncoders, KBins bins to their midpoints, and each row gets the model output
(sigmoid) and the predicted class; German rows are mapped back to the raw dataset's A-codes
(sex A91/A92 and the grouped categories, src/GC/Verify-GC-experiment-new2.py:364-414).  A code
outside an encoder's classes follows the reference per suite: Adult and German write the string
``f"{col}_{value}"`` and keep the row (src/AC/...-new2.py:373-374, src/GC/...-new2.py:355-356),
Bank drops the pair (src/BM/...-new2.py:360-368).  An ``.npz`` with the raw pairs is written next to
it (input of ``repair``).
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import pandas as pd


def _fmt_code(v) -> str:
    f = float(v)
    return str(int(f)) if f == int(f) else str(f)


def _decode_column(vals: np.ndarray, enc, name: str = "", keep_undecodable: bool = True) -> np.ndarray:
    """Encoded column -> decoded values.  An undecodable label code becomes ``f"{name}_{code}"``
    (``keep_undecodable``) or None (the row pair is dropped)."""
    if enc is None:
        return vals
    if hasattr(enc, "classes_"):            # LabelEncoder
        codes = np.rint(vals).astype(int)
        ok = (codes >= 0) & (codes < len(enc.classes_))
        out = np.empty(len(vals), dtype=object)
        out[ok] = enc.classes_[codes[ok]]
        out[~ok] = [f"{name}_{_fmt_code(v)}" for v in vals[~ok]] if keep_undecodable else None
        return out
    if hasattr(enc, "bin_edges_"):          # KBinsDiscretizer -> integer bin midpoint
        e = enc.bin_edges_[0]
        b = np.rint(vals).astype(int)
        out = np.empty(len(vals), dtype=object)
        inner = (b >= 0) & (b < len(e) - 1)
        bi = np.clip(b, 0, len(e) - 2)
        # int((start + end) / 2), the last edge past the last bin (src/AC/...-new2.py:360-370)
        out[:] = np.where(inner, np.trunc(0.5 * (e[bi] + e[bi + 1])), np.trunc(e[-1])).astype(np.int64)
        return out
    return vals


# German Credit: the fork maps the grouped categories and sex back to the dataset's A-codes
# (src/GC/Verify-GC-experiment-new2.py:364-414); the class column is called "decision" there
GC_REVERSE = {
    "credit_history": {"None/Paid": "A30", "Delay": "A33", "Other": "A34"},
    "savings": {"<500": "A61", "500+": "A63", "Unknown/None": "A65"},
    "employment": {"Unemployed": "A71", "1-4 years": "A72", "4+ years": "A74"},
    "status": {"<200": "A11", "200+": "A13", "None": "A14"},
}


def gc_reverse_map(df: pd.DataFrame) -> pd.DataFrame:
    """Decoded German rows -> the raw dataset's codes: sex 1 -> A91 (male), 0 -> A92 (female),
    grouped categories -> one representative A-code each (the reference's choice)."""
    out = df.copy()
    if "sex" in out.columns:
        sx = pd.to_numeric(out["sex"], errors="coerce")
        out["sex"] = np.where(sx == 1, "A91", np.where(sx == 0, "A92", out["sex"].astype(object)))
    for col, mp in GC_REVERSE.items():
        if col in out.columns:
            out[col] = out[col].map(lambda v, mp=mp: mp.get(v, v))
    return out


def export_counterexamples(preset: str, model: str, results: str, out: Optional[str] = None,
                           weights: str = "zoo") -> str:
    from .. import presets
    from ..data import tabular
    from ..models.zoo import get_model
    from .csv_report import read_csv

    pre = presets.get(preset)
    dom = pre.domain()
    mlp = get_model(model, weights=weights)
    rows = [r for r in read_csv(os.path.join(results, f"{model}.csv")) if r["Verification"] == "sat" and r["C1"]]

    def parse(s):
        return np.array([float(t) for t in s.replace("[", " ").replace("]", " ").split()])

    X = np.array([parse(r["C1"]) for r in rows]).reshape(-1, dom.n)
    XP = np.array([parse(r["C2"]) for r in rows]).reshape(-1, dom.n)
    pairs = np.stack([X, XP], axis=1).reshape(-1, dom.n)
    try:
        enc = tabular.load(pre.suite, allow_synthetic=False).encoders
    except Exception:
        enc = {}
    z = mlp.logits(pairs)
    keep_und = pre.suite != "bank"
    out_df = pd.DataFrame({name: _decode_column(pairs[:, i], enc.get(name), name, keep_und)
                           for i, name in enumerate(dom.names)})
    out_df["output"] = 0.5 * (1 + np.tanh(0.5 * z))
    label_col = "decision" if pre.suite == "german" else "prediction"
    out_df[label_col] = (z > 0).astype(int)
    keep = ~out_df[dom.names].isna().any(axis=1).to_numpy()
    keep = keep.reshape(-1, 2).all(axis=1).repeat(2)
    out_df = out_df[keep]
    if pre.suite == "german":
        out_df = gc_reverse_map(out_df)
    out = out or os.path.join(results, f"{model}-counterexample.csv")
    out_df.to_csv(out, index=False)
    np.savez(os.path.splitext(out)[0] + ".npz", x=X, xp=XP, y=np.maximum(z[0::2] > 0, z[1::2] > 0).astype(int))
    return out
