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


def _arr_fast(v: np.ndarray) -> str:
    """``str(np.asarray(v, float32))`` for the common case of an integer-valued vector that numpy
    prints in fixed notation ("[40.  0.  3.]", 75-column wrapping with a one-space hanging
    indent); anything else (exponent notation, fractions) goes through numpy itself."""
    v = np.asarray(v, dtype=np.float32)
    if v.ndim != 1 or v.size == 0 or not np.all(np.isfinite(v)) or np.any(v != np.round(v)):
        return _arr(v)
    nz = np.abs(v[v != 0])
    if nz.size and (nz.max() >= 1e8 or nz.min() < 1e-4 or nz.max() / nz.min() > 1000.0):
        return _arr(v)
    words = [f"{int(x)}." for x in v.tolist()]
    w = max(len(t) for t in words)
    words = [t.rjust(w) for t in words]
    out, line = "", " "
    last = len(words) - 1
    for i, word in enumerate(words):
        if len(line) + len(word) > 74 and len(line) > 1:
            out += line.rstrip() + "\n"
            line = " "
        line += word
        if i != last:
            line += " "
    out += line
    return "[" + out[1:] + "]"


_TEMPLATES: Dict[tuple, str] = {}


def _fixed_template(n: int, w: int) -> str:
    """str.format template of numpy's fixed-notation print of n integer-valued words of width w."""
    key = (n, w)
    if key not in _TEMPLATES:
        word = "{:>%d}." % (w - 1)
        out, line, llen = "", " ", 1
        for i in range(n):
            if llen + w > 74 and llen > 1:
                out += line.rstrip() + "\n"
                line, llen = " ", 1
            line += word
            llen += w
            if i != n - 1:
                line += " "
                llen += 1
        out += line
        _TEMPLATES[key] = "[" + out[1:] + "]"
    return _TEMPLATES[key]


def format_arrays(V: np.ndarray) -> List[str]:
    """``[_arr_fast(v) for v in V]`` for a 2-D block of vectors, vectorised per print width."""
    V = np.asarray(V, dtype=np.float32)
    k, n = V.shape
    out = [""] * k
    if k == 0:
        return out
    finite = np.all(np.isfinite(V), axis=1)
    Vs = np.where(np.isfinite(V), V, 0)
    integral = np.all(Vs == np.round(Vs), axis=1)
    A = np.abs(Vs)
    nzmax = A.max(axis=1)
    nzmin = np.where(A > 0, A, np.inf).min(axis=1)
    anynz = np.isfinite(nzmin)
    fixed = finite & integral & (~anynz | ((nzmax < 1e8) & (nzmin >= 1e-4) & (nzmax <= 1000.0 * nzmin)))
    I = Vs.astype(np.int64)
    lens = np.char.str_len(I.astype(str)).max(axis=1) + 1 if n else np.ones(k, np.int64)
    for w in np.unique(lens[fixed]).tolist():
        fmt = _fixed_template(n, int(w))
        sel = np.nonzero(fixed & (lens == w))[0]
        for i, row in zip(sel.tolist(), I[sel].tolist()):
            out[i] = fmt.format(*row)
    for i in np.nonzero(~fixed)[0].tolist():
        out[i] = _arr(V[i])
    return out


def _csv_field(x: str) -> str:
    return '"' + x.replace('"', '""') + '"' if ('\n' in x or '\r' in x or ',' in x or '"' in x) else x


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


    def write_packed(self, rows: np.ndarray, layout: List[int], n0: int, orig_acc: Optional[float],
                     native: bool = True) -> None:
        """Packed result rows (engine/runner.py:pack, ``layout`` = column indices of pos, verdict,
        h_attempt, h_success, b/s/st/h/t compressions, sv/s/hv/h/total times, c_check, v_accurate,
        pruned_acc, has_cex, c1 start, c2 start) -> CSV through the native formatter
        (csrc/csv_writer.cpp, ~1 us/row); same bytes as :meth:`write`."""
        if len(rows) == 0:
            return
        fmt = None
        if native:
            try:
                from .. import _C

                fmt = _C.format_partition_csv
            except ImportError:
                fmt = None
        if fmt is None:
            L = layout
            cols = {"partition_id": rows[:, L[0]].astype(np.int64) + 1, "verdict": rows[:, L[1]]}
            for k, name in enumerate(["h_attempt", "h_success", "b_comp", "s_comp", "st_comp", "h_comp", "t_comp",
                                      "sv_time", "s_time", "hv_time", "h_time", "total_time", "c_check",
                                      "v_accurate", "pruned_acc", "has_cex"]):
                cols[name] = rows[:, L[2 + k]]
            cols["c1"] = rows[:, L[18]:L[18] + n0]
            cols["c2"] = rows[:, L[19]:L[19] + n0]
            self.write_columns(cols, orig_acc)
            return
        c = self.counts
        data = fmt(np.ascontiguousarray(rows, dtype=np.float64), list(layout), int(n0),
                   [c["sat"], c["unsat"], c["unknown"]], orig_acc, _arr)
        v = rows[:, layout[1]].astype(np.int64)
        self.counts = {"sat": c["sat"] + int((v == 1).sum()), "unsat": c["unsat"] + int((v == 2).sum()),
                       "unknown": c["unknown"] + int(((v != 1) & (v != 2)).sum())}
        exists = os.path.isfile(self.path)
        with open(self.path, "ab") as fp:
            if not exists:
                fp.write((",".join(HEADER) + "\r\n").encode())
            fp.write(data)

    def write_columns(self, cols: Dict[str, np.ndarray], orig_acc: Optional[float]) -> None:
        """Columnar fast path of :meth:`write` (same bytes): ``cols`` holds per-partition arrays
        partition_id, verdict (0 unknown / 1 sat / 2 unsat), h_attempt, h_success, b_comp, s_comp,
        st_comp, h_comp, t_comp, sv_time, s_time, hv_time, h_time, total_time, c_check,
        v_accurate, pruned_acc, has_cex, c1 [n, n0], c2 [n, n0]."""
        n = len(cols["partition_id"])
        if n == 0:
            return
        v = np.asarray(cols["verdict"]).astype(np.int64)
        cs = self.counts["sat"] + np.cumsum(v == 1)
        cu = self.counts["unsat"] + np.cumsum(v == 2)
        ck = self.counts["unknown"] + np.cumsum(v == 0)
        self.counts = {"sat": int(cs[-1]), "unsat": int(cu[-1]), "unknown": int(ck[-1])}
        names = np.array(["unknown", "sat", "unsat"])[v].tolist()

        def ints(k):
            return [str(int(x)) for x in np.asarray(cols[k]).tolist()]

        def r4(k):
            return [repr(round(float(x), 4)) for x in np.asarray(cols[k]).tolist()]

        def raw(k):
            return [repr(float(x)) for x in np.asarray(cols[k]).tolist()]

        acc = '' if orig_acc is None else repr(round(orig_acc, 4))
        has = np.nonzero(np.asarray(cols["has_cex"]).astype(bool))[0]
        c1 = [''] * n
        c2 = [''] * n
        for dst, key in ((c1, "c1"), (c2, "c2")):
            for i, txt in zip(has.tolist(), format_arrays(np.asarray(cols[key])[has])):
                dst[i] = _csv_field(txt)
        colstr = [ints("partition_id"), names, [str(x) for x in cs.tolist()], [str(x) for x in cu.tolist()],
                  [str(x) for x in ck.tolist()], ints("h_attempt"), ints("h_success"), r4("b_comp"), r4("s_comp"),
                  r4("st_comp"), r4("h_comp"), r4("t_comp"), raw("sv_time"), raw("s_time"), raw("hv_time"),
                  raw("h_time"), raw("total_time"), ints("c_check"), ints("v_accurate"), [acc] * n,
                  r4("pruned_acc"), ['-'] * n, c1, c2]
        exists = os.path.isfile(self.path)
        with open(self.path, "a", newline='') as fp:
            if not exists:
                fp.write(",".join(HEADER) + "\r\n")
            fp.write("".join(",".join(row) + "\r\n" for row in zip(*colstr)))


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


def table_v_row_columns(model: str, pa: str, verdict: np.ndarray, h_attempt: np.ndarray, h_success: np.ndarray,
                        st_comp: np.ndarray, h_comp: np.ndarray, sv_time: np.ndarray, hv_time: np.ndarray,
                        total_time: np.ndarray, grid_size: int, wall: Optional[float] = None) -> Dict:
    """:func:`table_v_row` from per-partition columns (verdict 0 unknown / 1 sat / 2 unsat), so a
    multi-million-partition run never materialises per-partition record objects."""
    v = np.asarray(verdict).astype(np.int64)
    n = len(v)
    sat = int((v == 1).sum())
    uns = int((v == 2).sum())
    unk = n - sat - uns
    h = np.asarray(h_attempt).astype(bool)
    ver = "SAT" if sat else ("UNSAT" if n == grid_size and uns == n else "UNK")
    total = float(np.sum(total_time))
    wall = total if wall is None else wall
    return {
        "model": model, "PA": pa, "Ver": ver, "#P": n, "Grid": grid_size,
        "Cov%": round(100.0 * (sat + uns) / max(1, grid_size), 2), "SAT": sat, "UNSAT": uns, "UNK": unk,
        "#H": int(h.sum()), "#HS": int((np.asarray(h_success)[h] > 0).sum()),
        "C(S)": round(float(np.mean(st_comp)) if n else 0.0, 2),
        "C(H)": round(float(np.mean(np.asarray(h_comp)[h])) if h.any() else 0.0, 2),
        "SV": round(total and float(np.mean(sv_time)), 6),
        "HV": round(float(np.mean(np.asarray(hv_time)[h])) if h.any() else 0.0, 6),
        "Total": round(float(np.mean(total_time)) if n else 0.0, 6),
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
