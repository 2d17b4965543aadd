"""Partition-verdict store and hybrid routing (C27, K12).

Reference: ``partition_to_key`` / ``partition_results`` + ``find_partition_result_for_point``
(a linear scan over the stored boxes per test row) and ``hybrid_predict`` (route rows of ``sat``
partitions to the "fairer" model, others to the original; 3 single-row Keras predicts per row)
in src/AC/Verify-AC-experiment-new2.py:128-140,570-641.  Here the verdicts live in a dense
int8 table indexed by grid id, a point's partition is an O(n0) mixed-radix encode
(:meth:`Grid.encode`), and both models classify the whole test set in one batched forward each.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import numpy as np

from ..partition import Grid, processing_order

NOT_ATTEMPTED, V_UNKNOWN, V_SAT, V_UNSAT = -1, 0, 1, 2
_CODES = {"sat": V_SAT, "unsat": V_UNSAT, "unknown": V_UNKNOWN}


class VerdictTable:
    def __init__(self, grid: Grid):
        self.grid = grid
        self.table = np.full(grid.full_size, NOT_ATTEMPTED, dtype=np.int8)

    def set(self, grid_ids: np.ndarray, verdicts) -> None:
        v = np.array([_CODES[x] if isinstance(x, str) else int(x) for x in verdicts], dtype=np.int8)
        self.table[np.asarray(grid_ids, dtype=np.int64)] = v

    @classmethod
    def from_csv(cls, grid: Grid, csv_path: str, seed: int = 0) -> "VerdictTable":
        """Rebuild from a reference-format CSV (Partition_ID = position in the seeded order)."""
        from ..report.csv_report import read_csv

        t = cls(grid)
        order = processing_order(grid, seed=seed)
        rows = read_csv(csv_path)
        pos = np.array([int(r["Partition_ID"]) - 1 for r in rows], dtype=np.int64)
        t.set(order[pos], [r["Verification"] for r in rows])
        return t

    def lookup(self, X: np.ndarray) -> np.ndarray:
        ids = self.grid.encode(np.rint(np.asarray(X)).astype(np.int64))
        out = np.full(len(ids), NOT_ATTEMPTED, dtype=np.int8)
        ok = ids >= 0
        out[ok] = self.table[ids[ok]]
        return out

    def counts(self) -> Dict[str, int]:
        return {"sat": int((self.table == V_SAT).sum()), "unsat": int((self.table == V_UNSAT).sum()),
                "unknown": int((self.table == V_UNKNOWN).sum()),
                "not_attempted": int((self.table == NOT_ATTEMPTED).sum())}


def hybrid_predict(X: np.ndarray, table: VerdictTable, predict_orig, predict_fair) -> np.ndarray:
    """SAT partition -> fairer model; UNSAT / UNKNOWN / not attempted -> original model."""
    v = table.lookup(X)
    yo = np.asarray(predict_orig(X))
    yf = np.asarray(predict_fair(X))
    return np.where(v == V_SAT, yf, yo)


def case_breakdown(X: np.ndarray, table: VerdictTable) -> Dict[str, int]:
    """The fork's debug counters (src/AC/Verify-AC-experiment-new.py:594-620, 760-805): which
    branch of the hybrid predictor each test row takes."""
    v = table.lookup(X)
    return {"no_partition": int((v == NOT_ATTEMPTED).sum()), "sat_fairer": int((v == V_SAT).sum()),
            "unsat_original": int((v == V_UNSAT).sum()), "unknown_original": int((v == V_UNKNOWN).sum())}
