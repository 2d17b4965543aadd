"""Compact wire format of per-partition results for the rank-0 gather.

Round 1 shipped fixed-width float64 rows (≈376 B per Adult partition) with an ``all_gather``
to every rank.  Here a rank ships, per round, one byte buffer:

* header        int64 [5]: records, segments, SAT rows, n0, mask bytes per record (0 = none)
* segments      float64 [S, 5]: per verified chunk (count, t_sim+prune+bab, t_bab, t_heur,
                t_replay) -- the per-partition time columns are apportioned from these on
                rank 0 by :func:`engine.pipeline.derive_columns`, exactly as the producer would;
* records       22 B each (``REC``): flags (verdict 2 b | stage low 3 b | h_attempt | h_success |
                c_check | v_accurate | stage high bit, engine/stages.py codes), dead-neuron counts b/s/st/h/t (uint16), Pruned-acc
                numerator and the Pruned-F1 true / false positives (uint16), BaB node
                expansions (uint32);
* counterexamples, SAT partitions only: x [n0] and x' on the protected/relaxed dims only (every
                other dim of a confirmed pair equals x), int16 when the query domain (widened
                by tau) fits, else int32 -- 28 B per SAT pair for Adult;
* dead masks    optional (VerifyConfig.keep_masks, K6): every partition's final dead-neuron mask
                as a packed bitset, ceil(N/8) B (numpy.packbits order) -- the bitset all-gather of
                SURVEY §2.4.2 (26 B for AC-4's 201 neurons).

Partition positions are NOT shipped: rank 0 recomputes every rank's share of the round from
the seeded order (the same strided split the ranks used).  Verdicts alone travel as int8 in an
``all_gather`` when every rank needs them (residual work stealing).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

from ..engine.pipeline import ChunkRecords

VERDICTS = ("unknown", "sat", "unsat")
from ..engine.stages import STAGES
REC = np.dtype([("flags", "<u2"), ("b", "<u2"), ("s", "<u2"), ("st", "<u2"), ("h", "<u2"), ("t", "<u2"),
                ("agree", "<u2"), ("tp", "<u2"), ("fp", "<u2"), ("nodes", "<u4")])
assert REC.itemsize == 22


def verdict_codes(recs: ChunkRecords) -> np.ndarray:
    """int8 verdict per partition: 0 unknown, 1 sat, 2 unsat."""
    v = recs.core["verdict"]
    return np.select([v == "sat", v == "unsat"], [1, 2], 0).astype(np.int8)


def _cex_layout(q):
    """(x'-dims shipped, integer dtype) of the counterexample block for query ``q``."""
    dims = np.array(sorted(set(q.pa_idx) | set(q.ra_idx)), dtype=np.int64)
    lo, hi = q.domain.lo() - int(q.tau), q.domain.hi() + int(q.tau)
    narrow = int(max(np.abs(lo).max(), np.abs(hi).max())) <= np.iinfo(np.int16).max
    return dims, np.dtype(np.int16 if narrow else np.int32)


def encode(recs: ChunkRecords, q) -> np.ndarray:
    n0 = q.n
    c = recs.core
    n = len(c["verdict"])
    c = dict(c)
    for k in ("tp", "fp"):                       # older producers: no Pruned-F1 counts
        c.setdefault(k, np.zeros(n, dtype=np.int64))
    for k in ("b_cnt", "s_cnt", "st_cnt", "h_cnt", "t_cnt", "agree", "tp", "fp"):
        if n and int(np.max(c[k])) > 0xFFFF:
            raise OverflowError(f"{k} exceeds 16 bits")
    stage = np.array([STAGES.index(s) if s in STAGES else 0 for s in c["stage"]], dtype=np.uint16)
    flags = (verdict_codes(recs).astype(np.uint16) | ((stage & 7) << 2) | ((stage >> 3) << 9)
             | ((c["h_attempt"] > 0).astype(np.uint16) << 5)
             | ((c["h_success"] > 0).astype(np.uint16) << 6) | ((c["c_check"] > 0).astype(np.uint16) << 7)
             | ((c["v_accurate"] > 0).astype(np.uint16) << 8))
    rec = np.zeros(n, dtype=REC)
    rec["flags"] = flags
    rec["b"], rec["s"], rec["st"] = c["b_cnt"], c["s_cnt"], c["st_cnt"]
    rec["h"], rec["t"], rec["agree"] = c["h_cnt"], c["t_cnt"], c["agree"]
    rec["tp"], rec["fp"] = c["tp"], c["fp"]
    rec["nodes"] = np.minimum(c["nodes"], 0xFFFFFFFF)
    sat = c["verdict"] == "sat"
    dims, dt = _cex_layout(q)
    cex = np.concatenate([c["cex_x"][sat], c["cex_xp"][sat][:, dims]], axis=1).astype(dt)
    segs = np.asarray(recs.segments, dtype=np.float64).reshape(-1, 5)
    mb = c.get("mask_bits")
    nb = 0 if mb is None else int(mb.shape[1])
    head = np.array([n, len(segs), int(sat.sum()), n0, nb], dtype=np.int64)
    parts = [head.view(np.uint8), segs.reshape(-1).view(np.uint8), rec.view(np.uint8), cex.reshape(-1).view(np.uint8)]
    if nb:
        parts.append(np.ascontiguousarray(mb, dtype=np.uint8).reshape(-1))
    return np.concatenate(parts)


def decode(buf: np.ndarray, grid_ids: np.ndarray, orig_acc, n_neurons: int, sim_size: int, q) -> ChunkRecords:
    """Inverse of :func:`encode`; ``grid_ids`` = the partitions' grid ids (known to rank 0)."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    n, ns, nsat, n0, nb = (int(x) for x in buf[:HEAD].view(np.int64))
    o = HEAD
    segs = buf[o:o + 40 * ns].view(np.float64).reshape(ns, 5)
    o += 40 * ns
    rec = buf[o:o + REC.itemsize * n].view(REC)
    o += REC.itemsize * n
    dims, dt = _cex_layout(q)
    w = n0 + len(dims)
    cex = buf[o:o + dt.itemsize * w * nsat].view(dt).reshape(nsat, w).astype(np.int64)
    o += dt.itemsize * w * nsat
    masks = buf[o:o + n * nb].reshape(n, nb).copy() if nb else None
    if len(grid_ids) != n:
        raise ValueError(f"{n} records but {len(grid_ids)} grid ids")
    f = rec["flags"].astype(np.int64)
    verdict = np.array(VERDICTS, dtype=object)[f & 3].astype(str)
    sat = verdict == "sat"
    cx = np.zeros((n, n0), np.int64)
    cxp = np.zeros((n, n0), np.int64)
    cx[sat] = cex[:, :n0]
    xp = cex[:, :n0].copy()
    xp[:, dims] = cex[:, n0:]
    cxp[sat] = xp
    core = dict(grid_id=np.asarray(grid_ids, np.int64), verdict=verdict,
                stage=np.array(STAGES, dtype=object)[((f >> 2) & 7) | (((f >> 9) & 1) << 3)],
                h_attempt=(f >> 5) & 1, h_success=(f >> 6) & 1,
                b_cnt=rec["b"].astype(np.int64), s_cnt=rec["s"].astype(np.int64), st_cnt=rec["st"].astype(np.int64),
                h_cnt=rec["h"].astype(np.int64), t_cnt=rec["t"].astype(np.int64), agree=rec["agree"].astype(np.int64),
                tp=rec["tp"].astype(np.int64), fp=rec["fp"].astype(np.int64),
                nodes=rec["nodes"].astype(np.int64), c_check=(f >> 7) & 1, v_accurate=(f >> 8) & 1,
                cex_x=cx, cex_xp=cxp)
    if masks is not None:
        core["mask_bits"] = masks
    return ChunkRecords(core, orig_acc, segments=[tuple(s) for s in segs.tolist()], n_neurons=n_neurons,
                        sim_size=sim_size)


def bytes_per_partition(buf: np.ndarray, n: int) -> float:
    return len(buf) / max(1, n)


def empty(q) -> np.ndarray:
    return np.array([0, 0, 0, q.n, 0], dtype=np.int64).view(np.uint8).copy()


HEAD = 40   # header bytes (5 x int64)


def records_of(bufs: List[np.ndarray]) -> List[int]:
    return [int(np.ascontiguousarray(b[:8]).view(np.int64)[0]) for b in bufs]


def split_positions(positions: np.ndarray, world: int) -> List[np.ndarray]:
    """Every rank's strided share of ``positions`` (the split the ranks themselves use)."""
    return [positions[r::world] for r in range(world)]


def merge_rounds(parts: List[Tuple[np.ndarray, ChunkRecords]]) -> Tuple[np.ndarray, ChunkRecords]:
    """(positions, records) of several ranks -> one block sorted by position."""
    from ..engine.pipeline import concat_records

    parts = [(p, r) for p, r in parts if len(p)]
    if not parts:
        return np.zeros(0, np.int64), None
    pos = np.concatenate([p for p, _ in parts])
    recs = concat_records([r for _, r in parts])
    order = np.argsort(pos, kind="stable")
    core = {k: v[order] for k, v in recs.core.items()}
    # segments describe contiguous producer blocks: after the sort, carry the already derived
    # per-partition times over unchanged
    out = ChunkRecords(core, recs.orig_acc, segments=[(len(pos), 0.0, 0.0, 0.0, 0.0)], n_neurons=recs.n_neurons,
                       sim_size=recs.sim_size)
    for k in ("sv_time", "s_time", "hv_time", "h_time", "total_time"):
        out.cols[k] = recs.cols[k][order]
    out.segments = None
    return pos[order], out
