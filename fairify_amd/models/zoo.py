"""Model zoo: architectures of the reference's 53 Keras MLPs (C02).

Every model can be instantiated either with the shipped weights (converted once from the
reference's ``models/*/*.h5`` into ``fairify_amd/assets/zoo/*.npz`` by
``tools/import_zoo.py`` using the framework's own HDF5 reader) or with random
(glorot-uniform, Keras default) weights of the same shape — the synthetic benchmark setting.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

from .mlp import MLP, random_mlp

ASSET_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets", "zoo")

# name -> (suite, n_in, hidden widths)
ZOO: Dict[str, Tuple[str, int, Tuple[int, ...]]] = {}


def _reg(prefix: str, suite: str, n_in: int, table: Dict[int, Sequence[int]]):
    for k, h in table.items():
        ZOO[f"{prefix}-{k}"] = (suite, n_in, tuple(h))


_reg("AC", "adult", 13, {1: (16, 8), 2: (100,), 3: (50,), 4: (100, 100), 5: (64, 64), 6: (12, 12),
                         7: (64, 32, 16, 8, 4), 8: (5, 5), 9: (3, 3, 3, 3), 10: (5, 5, 5, 5),
                         11: (10, 10, 10, 10), 12: (5,) * 9})
_reg("BM", "bank", 16, {1: (64, 16), 2: (32, 16), 3: (100,), 4: (150, 100, 50), 5: (22, 10), 6: (9, 9),
                        7: (64, 64), 8: (64, 32, 16, 8, 4), 9: (30, 20), 10: (30, 20), 11: (30, 20),
                        12: (30, 20), 13: (30, 20)})
_reg("GC", "german", 20, {1: (50,), 2: (100,), 3: (9,), 4: (6, 4), 5: (64, 32, 16, 8, 4)})
_reg("CP", "compas", 6, {1: (16, 8), 11: (32, 32)})
_reg("CP", "compas12", 12, {k: (32, 32) for k in range(2, 11)})
ZOO["aCP-1-Old"] = ("compas12", 12, (32, 32))
_reg("DF", "default", 30, {k: (16, 16, 16) for k in range(1, 12)})

SUITE_PREFIX = {"adult": "AC", "bank": "BM", "german": "GC", "compas": "CP", "compas12": "CP", "default": "DF"}

# The models of the paper's Table V per suite (src/ presets iterate the model directory).
SUITE_MODELS: Dict[str, List[str]] = {
    "AC": [f"AC-{k}" for k in range(1, 13)],
    "BM": [f"BM-{k}" for k in range(1, 9)],
    "GC": [f"GC-{k}" for k in range(1, 6)],
    "CP": ["CP-1", "CP-11"] + [f"CP-{k}" for k in range(2, 11)],
    "DF": [f"DF-{k}" for k in range(1, 12)],
}


def asset_path(name: str) -> str:
    return os.path.join(ASSET_DIR, f"{name}.npz")


def has_weights(name: str) -> bool:
    return os.path.isfile(asset_path(name))


def get_model(name: str, weights: str = "zoo", seed: int = 0) -> MLP:
    """Instantiate a zoo model.  ``weights``: 'zoo' (shipped weights; falls back to an error if
    absent), 'random' (glorot-uniform with ``seed``), or a path to a ``.h5``/``.npz`` file."""
    if name not in ZOO:
        raise KeyError(f"unknown zoo model {name}")
    suite, n_in, hidden = ZOO[name]
    if weights == "random":
        # derive a per-model stream so suites are reproducible and models differ
        sub = (seed * 1000003 + sum(ord(c) * (i + 1) for i, c in enumerate(name))) % (2 ** 31)
        return random_mlp(n_in, hidden, seed=sub, name=name)
    if weights == "zoo":
        p = asset_path(name)
        if not os.path.isfile(p):
            raise FileNotFoundError(f"no shipped weights for {name} ({p}); use weights='random'")
        m = MLP.load_npz(p)
        m.name = name
        return m
    if weights.endswith(".h5"):
        from .keras_io import load_keras_h5

        return load_keras_h5(weights, name=name)
    return MLP.load_npz(weights)


def suite_of(name: str) -> str:
    return ZOO[name][0]
