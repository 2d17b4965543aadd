"""Keras ``.h5`` model zoo I/O (C05: reference ``src/AC/Verify-AC.py:92-99``; the fork's
Dense-only filter ``src/BM/Verify-BM-experiment.py:103-122``).

Weights are read with the framework's own HDF5 reader; only ``Dense`` layers that carry a
kernel are kept, in ``layer_names`` order.
"""
from __future__ import annotations

import json
import os
import re
from typing import List, Optional

import numpy as np

from .hdf5 import H5File
from .mlp import MLP


def _natural_key(s: str):
    return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", s)]


def load_keras_h5(path: str, name: Optional[str] = None) -> MLP:
    f = H5File(path)
    root = "model_weights" if "model_weights" in f.keys("/") else "/"
    attrs = f.attrs(root)
    layer_names = attrs.get("layer_names")
    if layer_names is None:
        layer_names = sorted(f.keys(root), key=_natural_key)
    ws, bs = [], []
    for ln in list(layer_names):
        gpath = f"{root}/{ln}".replace("//", "/")
        gattrs = f.attrs(gpath)
        wnames = list(gattrs.get("weight_names", []))
        kern = [w for w in wnames if w.split("/")[-1].startswith("kernel")]
        bias = [w for w in wnames if w.split("/")[-1].startswith("bias")]
        if not kern:
            continue  # Dropout / InputLayer / activation-only layers
        ws.append(np.asarray(f.dataset(f"{gpath}/{kern[0]}"), dtype=np.float32))
        if bias:
            bs.append(np.asarray(f.dataset(f"{gpath}/{bias[0]}"), dtype=np.float32))
        else:
            bs.append(np.zeros(ws[-1].shape[1], dtype=np.float32))
    if name is None:
        name = os.path.splitext(os.path.basename(path))[0]
    return MLP(ws, bs, name=name)


def model_config(path: str) -> Optional[dict]:
    f = H5File(path)
    cfg = f.attrs("/").get("model_config")
    if cfg is None:
        return None
    if isinstance(cfg, bytes):
        cfg = cfg.decode()
    return json.loads(cfg)


def activations_from_config(cfg: dict) -> List[str]:
    """Activation of every Dense layer in a Keras ``model_config`` (for validation)."""
    layers = cfg.get("config", {})
    if isinstance(layers, dict):
        layers = layers.get("layers", [])
    return [l["config"].get("activation", "linear") for l in layers if l.get("class_name") == "Dense"]
