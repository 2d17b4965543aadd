"""Result writers: the reference's 24-column per-partition CSV and the Table-V summary.

* per-partition CSV — same header, column order and value formatting as the reference
  (``src/AC/Verify-AC.py:277-315``): cumulative SAT/UNSAT/UNK counts, compressions rounded
  to 4 digits, ``Acc-dec`` always ``'-'``, counterexamples as NumPy float32 array reprs;
* ``summary.json`` / Table-V row per model (the paper's aggregation was
  offline): #P, coverage, verdict counts, heuristic attempts/successes,
  average compressions and times, partitions/s.
"""
from __future__ import annotations

import csv
import json
import os
from typing import Dict, Iterable, List, Optional

import numpy as np

HEADER = ['Partition_ID', 'Verification', 'SAT_count', 'UNSAT_count', 'UNK_count', 'h_attempt', 'h_success',
          'B_compression', 'S_compression', 'ST_compression', 'H_compression', 'T_compression', 'SV-time',
          'S-time', 'HV-Time', 'H-Time', 'Total-Time', 'C-check', 'V-accurate', 'Original-acc', 'Pruned-acc',
          'Acc-dec', 'C1', 'C2']


def _arr(a: Optional[np.ndarray]) -> str:
    if a is None:
        return ''
    return str(np.asarray(a, dtype=np.float32))


class PartitionCSV:
    """Append-mode writer with running counts (one file per model, like the reference)."""

    def __init__(self, path: str, resume: bool = False):
        self.path = path
        self.counts = {"sat": 0, "unsat": 0, "unknown": 0}
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        if os.path.exists(path) and resume:
            with open(path, newline='') as f:
                rows = list(csv.reader(f))[1:]
            for r in rows:
                if r:
                    self.counts = {"sat": int(r[2]), "unsat": int(r[3]), "unknown": int(r[4])}
        elif os.path.exists(path):
            os.remove(path)

    def write(self, records: Iterable) -> None:
        exists = os.path.isfile(self.path)
        with open(self.path, "a", newline='') as fp:
            wr = csv.writer(fp, dialect='excel')
            if not exists:
                wr.writerow(HEADER)
            for r in records:
                self.counts[r.verdict] += 1
                wr.writerow([
                    r.partition_id, r.verdict, self.counts["sat"], self.counts["unsat"], self.counts["unknown"],
                    r.h_attempt, r.h_success, round(r.b_comp, 4), round(r.s_comp, 4), round(r.st_comp, 4),
                    round(r.h_comp, 4), round(r.t_comp, 4), r.sv_time, r.s_time, r.hv_time, r.h_time,
                    r.total_time, r.c_check, r.v_accurate,
                    '' if r.orig_acc is None else round(r.orig_acc, 4), round(r.pruned_acc, 4), '-',
                    _arr(r.c1), _arr(r.c2),
                ])


def read_csv(path: str) -> List[Dict[str, str]]:
    with open(path, newline='') as f:
        return list(csv.DictReader(f))


def table_v_row(model: str, pa: str, records: List, grid_size: int, wall: Optional[float] = None) -> Dict:
    """One row of the paper's Table V recomputed from per-partition records."""
    n = len(records)
    sat = sum(1 for r in records if r.verdict == "sat")
    uns = sum(1 for r in records if r.verdict == "unsat")
    unk = n - sat - uns
    h = [r for r in records if r.h_attempt]
    ver = "SAT" if sat else ("UNSAT" if n == grid_size and uns == n else "UNK")
    total = sum(r.total_time for r in records)
    wall = total if wall is None else wall
    return {
        "model": model, "PA": pa, "Ver": ver, "#P": n, "Grid": grid_size,
        "Cov%": round(100.0 * (sat + uns) / max(1, grid_size), 2), "SAT": sat, "UNSAT": uns, "UNK": unk,
        "#H": len(h), "#HS": sum(1 for r in h if r.h_success),
        "C(S)": round(float(np.mean([r.st_comp for r in records])) if n else 0.0, 2),
        "C(H)": round(float(np.mean([r.h_comp for r in h])) if h else 0.0, 2),
        "SV": round(total and float(np.mean([r.sv_time for r in records])), 6),
        "HV": round(float(np.mean([r.hv_time for r in h])) if h else 0.0, 6),
        "Total": round(float(np.mean([r.total_time for r in records])) if n else 0.0, 6),
        "partitions_per_s": round(n / wall, 3) if wall else 0.0,
        "decided_per_s": round((sat + uns) / wall, 3) if wall else 0.0,
        "verified_of_attempted%": round(100.0 * (sat + uns) / max(1, n), 2),
        "wall_s": round(wall, 3),
    }


def format_table(rows: List[Dict]) -> str:
    cols = ["model", "PA", "Ver", "#P", "Grid", "Cov%", "SAT", "UNSAT", "UNK", "#H", "#HS", "C(S)", "C(H)",
            "Total", "partitions_per_s"]
    w = {c: max(len(c), *(len(str(r.get(c, ""))) for r in rows)) if rows else len(c) for c in cols}
    lines = ["  ".join(c.rjust(w[c]) for c in cols)]
    for r in rows:
        lines.append("  ".join(str(r.get(c, "")).rjust(w[c]) for c in cols))
    return "\n".join(lines)


def write_summary(path: str, rows: List[Dict], extra: Optional[Dict] = None) -> None:
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "w") as f:
        json.dump({"models": rows, **(extra or {})}, f, indent=2)
