"""Fine-tuning on synthetic (counterexample-derived) data with early stopping (C31, GC/BM).

Reference: ``src/GC/new_model.py:8-58`` and ``src/BM/new_model.py:8-40`` -- load a trained
model, read a synthetic CSV (LLM/CTGAN-generated rows labelled by the model), label-encode the
categorical columns with FRESH ``LabelEncoder``s fitted on that CSV, hold out 15 %
(``train_test_split(test_size=0.15, random_state=42)``), then Keras ``fit`` with Adam(lr 5e-4),
binary cross-entropy, batch 32, up to 100 epochs and ``EarlyStopping(monitor='val_loss',
patience=3, restore_best_weights=True)``; the result is saved as a new zoo entry (GC-8, BM-6).

Re-implemented on ``torch.nn`` (CPU or ROCm): logits + ``BCEWithLogitsLoss`` (the Keras model
ends in a sigmoid), Adam with Keras' epsilon (1e-7), per-epoch shuffling like ``fit``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..models.mlp import MLP

# categorical columns the reference label-encodes per suite, and the label column
SUITE_SPECS: Dict[str, Dict] = {
    "german": dict(label="credit", categorical=[
        "status", "credit_history", "purpose", "savings", "employment", "other_debtors", "property",
        "installment_plans", "housing", "skill_level", "telephone", "foreign_worker"]),
    "bank": dict(label="y", categorical=[
        "job", "marital", "education", "default", "housing", "loan", "contact", "month", "day_of_week",
        "emp.var.rate", "duration", "campaign", "pdays", "previous", "poutcome", "age"]),
}


@dataclass
class FinetuneResult:
    model: MLP
    epochs_run: int
    best_epoch: int
    val_loss: List[float]
    val_acc: float
    train_rows: int
    val_rows: int


def encode_synthetic(df, label: str, categorical: Sequence[str]):
    """``X = df.drop(columns=[label])``; fresh LabelEncoder per categorical column (fit on this
    CSV, as the reference does); returns (X float64, y int)."""
    from sklearn.preprocessing import LabelEncoder

    X = df.drop(columns=[label]).copy()
    for c in categorical:
        if c in X.columns:
            X[c] = LabelEncoder().fit_transform(X[c])
    return X.to_numpy(dtype=np.float64), df[label].to_numpy().astype(np.int64)


def finetune(mlp: MLP, X: np.ndarray, y: np.ndarray, lr: float = 5e-4, batch: int = 32, epochs: int = 100,
             patience: int = 3, test_size: float = 0.15, split_seed: int = 42, seed: int = 0,
             device: str = "cpu", name: Optional[str] = None) -> FinetuneResult:
    """Keras-``fit`` equivalent with EarlyStopping(val_loss, patience, restore_best_weights)."""
    from sklearn.model_selection import train_test_split

    if X.shape[1] != mlp.n_in:
        raise ValueError(f"data has {X.shape[1]} features, the model {mlp.n_in}")
    Xtr, Xva, ytr, yva = train_test_split(X, y, test_size=test_size, random_state=split_seed)
    torch.manual_seed(seed)
    net = mlp.to_torch(device)
    opt = torch.optim.Adam(net.parameters(), lr=lr, eps=1e-7)
    lossf = torch.nn.BCEWithLogitsLoss()
    xt = torch.as_tensor(Xtr, dtype=torch.float32, device=device)
    yt = torch.as_tensor(ytr, dtype=torch.float32, device=device)
    xv = torch.as_tensor(Xva, dtype=torch.float32, device=device)
    yv = torch.as_tensor(yva, dtype=torch.float32, device=device)
    g = torch.Generator(device="cpu").manual_seed(seed)
    best, best_ep, best_state, wait = float("inf"), -1, None, 0
    hist: List[float] = []
    ep = 0
    for ep in range(epochs):
        net.train()
        perm = torch.randperm(len(xt), generator=g).to(device)
        for s in range(0, len(xt), batch):
            idx = perm[s:s + batch]
            opt.zero_grad()
            loss = lossf(net(xt[idx]).reshape(-1), yt[idx])
            loss.backward()
            opt.step()
        net.eval()
        with torch.no_grad():
            vl = float(lossf(net(xv).reshape(-1), yv))
        hist.append(vl)
        if vl < best:
            best, best_ep, wait = vl, ep, 0
            best_state = {k: v.detach().clone() for k, v in net.state_dict().items()}
        else:
            wait += 1
            if wait >= patience:
                break
    if best_state is not None:
        net.load_state_dict(best_state)
    out = MLP.from_torch(net, name=name or f"{mlp.name}-ft")
    with torch.no_grad():
        acc = float(((net(xv).reshape(-1) > 0).float() == yv).float().mean()) if len(xv) else 0.0
    return FinetuneResult(out, ep + 1, best_ep + 1, hist, acc, len(xt), len(xv))


def finetune_csv(mlp: MLP, csv_path: str, suite: str, **kw) -> FinetuneResult:
    import pandas as pd

    spec = SUITE_SPECS[suite]
    df = pd.read_csv(csv_path)
    X, y = encode_synthetic(df, spec["label"], spec["categorical"])
    return finetune(mlp, X, y, **kw)
