"""Group-fairness metrics of a classifier's predictions (C28; AIF360-equivalent, K10).

The fork computes them with AIF360's ``ClassificationMetric`` / ``BinaryLabelDatasetMetric``
(src/AC/Verify-AC-experiment-new.py:482-542; src/AC/detect_bias.py:51-116).  AIF360 is not
available here, so the definitions are re-implemented directly (privileged group = PA == 1):

* DI  = P(yhat=1 | unpriv) / P(yhat=1 | priv)                (disparate impact)
* SPD = P(yhat=1 | unpriv) - P(yhat=1 | priv)                (statistical parity difference)
* EOD = TPR_unpriv - TPR_priv                                (equal opportunity difference)
* AOD = ((FPR_u - FPR_p) + (TPR_u - TPR_p)) / 2              (average odds difference)
* ERD = ERR_u - ERR_p                                        (error rate difference)
* CNT = 1 - mean_i |yhat_i - mean(yhat over the 5 nearest neighbours of x_i, incl. itself)|
* TI  = generalized entropy index alpha=1 of b_i = yhat_i - y_i + 1  (Theil index)

The consistency kNN (the only super-linear part) runs as tiled distance GEMMs + top-k on the
device (torch on ROCm, i.e. hipBLASLt GEMMs; chunked so [chunk, n] distances stay small).
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch


def _rate(mask: np.ndarray, num: np.ndarray) -> float:
    d = mask.sum()
    return float(num[mask].sum() / d) if d else float("nan")


def group_metrics(y_true: np.ndarray, y_pred: np.ndarray, protected: np.ndarray, privileged_value=1) -> Dict[str, float]:
    y_true = np.asarray(y_true).astype(int)
    y_pred = np.asarray(y_pred).astype(int)
    priv = np.asarray(protected) == privileged_value
    unp = ~priv
    pos_u = _rate(unp, y_pred == 1)
    pos_p = _rate(priv, y_pred == 1)
    tpr_u = _rate(unp & (y_true == 1), y_pred == 1)
    tpr_p = _rate(priv & (y_true == 1), y_pred == 1)
    fpr_u = _rate(unp & (y_true == 0), y_pred == 1)
    fpr_p = _rate(priv & (y_true == 0), y_pred == 1)
    err_u = _rate(unp, y_pred != y_true)
    err_p = _rate(priv, y_pred != y_true)
    return {
        "DI": pos_u / pos_p if pos_p else float("nan"),
        "SPD": pos_u - pos_p,
        "EOD": tpr_u - tpr_p,
        "AOD": 0.5 * ((fpr_u - fpr_p) + (tpr_u - tpr_p)),
        "ERD": err_u - err_p,
    }


def consistency(X: np.ndarray, y_pred: np.ndarray, k: int = 5, device=None, chunk: int = 4096,
                method: str = "auto") -> float:
    """AIF360 ``consistency()`` (kNN over features, neighbours include the point itself).

    Integer features make equidistant neighbours common, so the k-set depends on tie-breaking.
    AIF360 uses ``NearestNeighbors(algorithm='ball_tree')``: ``method='ball_tree'`` (the default
    via ``auto`` when scikit-learn is importable and X has at most 200 000 rows) reproduces it
    exactly -- AC-3's logged "Original CNT: 0.8890" (AC-3.ipynb:2086); the GEMM + top-k path
    (``method='gemm'``, device-resident, for large X) breaks ties by index and gives 0.8886."""
    if method in ("auto", "ball_tree") and len(X) <= 200_000:
        try:
            from sklearn.neighbors import NearestNeighbors
        except Exception:
            NearestNeighbors = None
        if NearestNeighbors is not None:
            Xn = np.asarray(X, dtype=np.float64)
            yn = np.asarray(y_pred, dtype=np.float64)
            _, idx = NearestNeighbors(n_neighbors=k, algorithm="ball_tree").fit(Xn).kneighbors(Xn)
            return float(1.0 - np.mean(np.abs(yn - yn[idx].mean(axis=1))))
    dev = torch.device(device) if device is not None else torch.device("cpu")
    Xt = torch.as_tensor(np.asarray(X, dtype=np.float32), device=dev)
    yp = torch.as_tensor(np.asarray(y_pred, dtype=np.float32), device=dev)
    n = Xt.shape[0]
    if dev.type == "cuda" and method in ("auto", "gemm", "device"):
        from ..ops import use_hip

        if use_hip(Xt):
            from ..ops import hip as H

            if k in H.KNN_K and k <= n and Xt.shape[1] <= 64:
                # K10 on the device: fa_knn_kernel (exact differences, ties to the lower index)
                idx, _ = H.knn(Xt, k)
                return float(1.0 - (yp - yp[idx.long()].mean(1)).abs().mean())
    sq = (Xt * Xt).sum(1)
    acc = 0.0
    for s in range(0, n, chunk):
        q = Xt[s:s + chunk]
        d = sq[s:s + chunk, None] - 2.0 * (q @ Xt.T) + sq[None, :]
        # exact self-distance 0 (avoid fp cancellation noise moving the point itself out of the k set)
        ar = torch.arange(q.shape[0], device=dev)
        d[ar, s + ar] = -1.0
        idx = d.topk(k, dim=1, largest=False).indices
        acc += float((yp[s:s + chunk] - yp[idx].mean(1)).abs().sum())
    return 1.0 - acc / max(1, n)


def theil_index(y_true: np.ndarray, y_pred: np.ndarray) -> float:
    b = np.asarray(y_pred, dtype=np.float64) - np.asarray(y_true, dtype=np.float64) + 1.0
    mu = b.mean()
    r = b / mu
    with np.errstate(divide="ignore", invalid="ignore"):
        t = np.where(r > 0, r * np.log(r), 0.0)
    return float(t.mean())


def all_metrics(X: np.ndarray, y_true: np.ndarray, y_pred: np.ndarray, pa_index: int, device=None) -> Dict[str, float]:
    from sklearn.metrics import accuracy_score, f1_score

    out = {"accuracy": float(accuracy_score(y_true, y_pred)), "f1": float(f1_score(y_true, y_pred, zero_division=0))}
    out.update(group_metrics(y_true, y_pred, X[:, pa_index]))
    out["CNT"] = consistency(X, y_pred, device=device)
    out["TI"] = theil_index(y_true, y_pred)
    return out
