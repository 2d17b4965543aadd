"""Preset runner: data-parallel verification of a model list with checkpoint/resume.

Reference flow: ``for model_file in os.listdir(model_dir): for p in p_list: ...`` with one CSV
append per partition and a per-model hard timeout (src/AC/Verify-AC.py:78-320).  Here:

* the seeded processing order is split into *rounds*; in every round the ranks share the round's
  block of the order through a dynamic unit queue (``balance="queue"``, the default with several
  ranks): every host thread of every rank claims the next unit of partitions from an atomic counter
  in the rendezvous store (``store.add``) until the round is exhausted, so a rank that drew
  expensive partitions simply claims fewer units -- the heavy tail of the BaB (SURVEY §2.4.2 work
  stealing, §7.5) is balanced without a cost model; ``balance="strided"`` keeps round 1's fixed
  strided shares;
* per-partition records are packed into fixed-width rows and ``all_gather``-ed (RCCL) to rank 0,
  which appends them to the reference-format CSV in processing order and checkpoints the set
  of finished positions (``state/<model>.npz``) so ``--resume`` skips them;
* the hard timeout is a global decision (``all_reduce(MAX)`` of elapsed time), so all ranks
  stop at the same round;
* rank 0 prints/writes the Table-V row of every model (``summary.json``).
"""
from __future__ import annotations

import json
import os
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import asdict, replace
from typing import Dict, List, Optional

import numpy as np

from ..models.zoo import get_model
from ..ops.backend import Backend
from ..parallel import dist as D
from ..parallel import wire
from ..partition import processing_order
from ..presets import Preset
from ..report.csv_report import PartitionCSV, format_table, table_v_row_columns, write_summary
from ..utils import faults, heap
from ..utils.timer import StageTimer
from .stages import STAGES as _STAGES
from .pipeline import STAGE_NODE_COLS, PartitionRecord, StreamPool, VerifyConfig, concat_records, verify_chunk

VCODE = {"sat": 1, "unsat": 2, "unknown": 0}
VNAME = {v: k for k, v in VCODE.items()}
STAGES = list(_STAGES)
_SCALARS = ["h_attempt", "h_success", "b_comp", "s_comp", "st_comp", "h_comp", "t_comp", "sv_time", "s_time",
            "hv_time", "h_time", "total_time", "c_check", "v_accurate", "pruned_acc", "nodes"]


def pack(records, positions: np.ndarray, n0: int) -> np.ndarray:
    """Fixed-width float64 rows [pos, grid_id, verdict, stage, scalars..., has_cex, c1[n0], c2[n0]]:
    the input of the native CSV formatter on rank 0 (never sent over the wire; ranks ship
    :mod:`parallel.wire` buffers)."""
    w = 4 + len(_SCALARS) + 1 + 2 * n0
    out = np.zeros((len(records), w), dtype=np.float64)
    cols = records.cols
    out[:, 0] = positions
    out[:, 1] = cols["grid_id"]
    out[:, 2] = np.select([cols["verdict"] == "sat", cols["verdict"] == "unsat"], [1, 2], 0)
    out[:, 3] = [STAGES.index(x) if x in STAGES else 0 for x in cols["stage"]]
    for k, name in enumerate(_SCALARS):
        out[:, 4 + k] = cols[name]
    sat = cols["verdict"] == "sat"
    out[:, 4 + len(_SCALARS)] = sat
    out[sat, 5 + len(_SCALARS):5 + len(_SCALARS) + n0] = cols["cex_x"][sat]
    out[sat, 5 + len(_SCALARS) + n0:] = cols["cex_xp"][sat]
    return out


def unpack(rows: np.ndarray, n0: int, orig_acc: Optional[float]) -> List[PartitionRecord]:
    """Packed rows -> per-partition record objects (the per-record CSV writer's input)."""
    recs = []
    for row in rows:
        kw = {name: row[4 + k] for k, name in enumerate(_SCALARS)}
        for name in ("h_attempt", "h_success", "c_check", "v_accurate", "nodes"):
            kw[name] = int(kw[name])
        has = row[4 + len(_SCALARS)] > 0
        c1 = row[5 + len(_SCALARS):5 + len(_SCALARS) + n0].astype(np.float32) if has else None
        c2 = row[5 + len(_SCALARS) + n0:].astype(np.float32) if has else None
        recs.append(PartitionRecord(partition_id=int(row[0]) + 1, grid_id=int(row[1]), verdict=VNAME[int(row[2])],
                                    stage=STAGES[int(row[3])], c1=c1, c2=c2, orig_acc=orig_acc, **kw))
    return recs


def columns(rows: np.ndarray, n0: int) -> Dict[str, np.ndarray]:
    """Packed rows -> the per-partition columns of :meth:`PartitionCSV.write_columns`."""
    c = {name: rows[:, 4 + k] for k, name in enumerate(_SCALARS)}
    c["partition_id"] = rows[:, 0].astype(np.int64) + 1
    c["grid_id"] = rows[:, 1].astype(np.int64)
    c["verdict"] = rows[:, 2].astype(np.int64)
    c["stage"] = rows[:, 3].astype(np.int64)
    c["has_cex"] = rows[:, 4 + len(_SCALARS)] > 0
    c["c1"] = rows[:, 5 + len(_SCALARS):5 + len(_SCALARS) + n0].astype(np.float32)
    c["c2"] = rows[:, 5 + len(_SCALARS) + n0:].astype(np.float32)
    return c


def csv_layout(n0: int) -> List[int]:
    """Column indices of the packed rows for PartitionCSV.write_packed."""
    ix = {name: 4 + k for k, name in enumerate(_SCALARS)}
    return [0, 2, ix["h_attempt"], ix["h_success"], ix["b_comp"], ix["s_comp"], ix["st_comp"], ix["h_comp"],
            ix["t_comp"], ix["sv_time"], ix["s_time"], ix["hv_time"], ix["h_time"], ix["total_time"],
            ix["c_check"], ix["v_accurate"], ix["pruned_acc"], 4 + len(_SCALARS), 5 + len(_SCALARS),
            5 + len(_SCALARS) + n0]


def _save_done(path: str, done: np.ndarray) -> None:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tmp = path + ".tmp.npz"
    np.savez(tmp, done_bits=np.packbits(done), total=np.int64(len(done)))
    os.replace(tmp, path)


def _load_done(path: str, total: int) -> np.ndarray:
    z = np.load(path)
    done = np.zeros(total, dtype=bool)
    if "done_bits" in z:
        bits = np.unpackbits(z["done_bits"])[:int(z["total"])].astype(bool)
        done[:min(total, len(bits))] = bits[:total]
    else:                                           # older checkpoints: list of positions
        pos = z["done"].astype(np.int64)
        done[pos[pos < total]] = True
    return done


def _write_round(writer: PartitionCSV, rows: np.ndarray, n0: int, acc, done: np.ndarray, state_path: str) -> None:
    """CSV rows of one round, then the checkpoint that covers them (so resume never duplicates)."""
    writer.write_packed(rows, csv_layout(n0), n0, acc)
    done[rows[:, 0].astype(np.int64)] = True
    _save_done(state_path, done)


_TABLE_COLS = ("verdict", "h_attempt", "h_success", "st_comp", "h_comp", "sv_time", "hv_time", "total_time", "stage")


def model_accuracy(mlp, suite: str, seed: int = 0, with_source: bool = False):
    """``Original-acc`` column: test accuracy on the suite's dataset (real when available).
    ``with_source``: returns ``(acc, source)``, source "reference-data" or "synthetic" (the
    reference's CSVs are absent, e.g. on the GPU box: the number is then NOT the paper's
    column and is labelled as such in summary.json)."""
    from ..data import tabular

    try:
        ds = tabular.load(suite, seed=seed)
    except Exception:
        return (None, None) if with_source else None
    if ds.X_test.shape[1] != mlp.n_in:
        return (None, None) if with_source else None
    acc = float(np.mean(mlp.predict(ds.X_test) == ds.y_test))
    if with_source:
        return acc, ("synthetic" if getattr(ds, "synthetic", False) else "reference-data")
    return acc


def _claim_fn(info: D.DistInfo):
    """Atomic unit counter shared by all ranks (the process group's rendezvous store: TCPStore
    ``add`` is one round trip, thread-safe); single process: a local counter."""
    if info.initialized:
        import torch.distributed.distributed_c10d as c10d

        store = c10d._get_default_store()
        return lambda key: int(store.add(key, 1)) - 1
    import itertools
    import threading

    counters: Dict[str, "itertools.count"] = {}
    lock = threading.Lock()

    def claim(key):
        with lock:
            return next(counters.setdefault(key, itertools.count()))

    return claim


def queue_unit_size(n_round: int, world: int, workers: int, chunk: int) -> int:
    """Partitions per claimed unit: about 4 units per host thread of every rank (enough slack for
    the dynamic queue to even out heavy partitions), never more than a chunk."""
    return int(max(1, min(chunk, -(-n_round // max(1, 4 * world * workers)))))


def _pack_positions(pos: np.ndarray, buf: np.ndarray) -> np.ndarray:
    """Prefix a rank's wire buffer with the (claimed, hence not recomputable) positions it verified."""
    pos = np.ascontiguousarray(pos, dtype=np.int64)
    head = np.array([pos.size], dtype=np.int64)
    return np.concatenate([head.view(np.uint8), pos.view(np.uint8), np.asarray(buf, dtype=np.uint8).reshape(-1)])


def _unpack_positions(b: np.ndarray):
    n = int(np.frombuffer(b[:8].tobytes(), dtype=np.int64)[0])
    pos = np.frombuffer(b[8:8 + 8 * n].tobytes(), dtype=np.int64).copy()
    return pos, b[8 + 8 * n:]


def _round_positions(todo: np.ndarray, r: int, per_round: int, world: int) -> List[np.ndarray]:
    """Every rank's positions of round ``r`` (rank k verifies ``todo[k::world]`` in rounds of
    ``per_round``); rank 0 uses this instead of receiving positions over the wire."""
    return [todo[k::world][r * per_round:(r + 1) * per_round] for k in range(world)]


def _residual_pass(be, mlp, q, grid, order, round_pos: np.ndarray, codes: np.ndarray, cfg: VerifyConfig,
                   escalate: int, acc, info: D.DistInfo, timer, budget: float):
    """Residual re-distribution ("work stealing"): the UNKNOWN partitions of the
    round -- wherever they fell -- are re-sharded evenly over the ranks and retried with an
    escalated node budget.  Every rank holds the round's int8 verdicts (``codes``, aligned with
    ``round_pos``), so the split needs no extra coordination.  Returns (positions, records) of
    the retried partitions on rank 0 (``None`` elsewhere)."""
    unk = round_pos[codes == VCODE["unknown"]] if len(round_pos) else np.zeros(0, np.int64)
    if unk.size == 0 or budget <= 0:
        return None
    shares = wire.split_positions(unk, info.world)
    share = shares[info.rank]
    c2 = replace(cfg, node_budget=cfg.node_budget * escalate,
                 heuristic_node_budget=cfg.heuristic_node_budget * escalate)
    buf = wire.empty(q)
    if len(share):
        recs = verify_chunk(be, mlp, q, grid, order[share], c2, orig_acc=acc, time_budget=budget, timer=timer)
        buf = wire.encode(recs, q)
    bufs = D.gather_bytes(info, buf)
    if not info.is_main:
        return None
    parts = [(sh, wire.decode(b, order[sh], acc, mlp.n_neurons, cfg.sim_size, q)) for sh, b in zip(shares, bufs)]
    return wire.merge_rounds(parts)


def _replace(pos: np.ndarray, recs, new_pos: np.ndarray, new_recs) -> None:
    """Overwrite the rows of ``recs`` (sorted by ``pos``) at ``new_pos`` with ``new_recs``."""
    idx = np.searchsorted(pos, new_pos)
    for k, v in new_recs.cols.items():
        recs.cols[k][idx] = v


class _MetricsCSV:
    """Per-partition metrics CSV of the fork's experiment drivers: one row per verified
    partition with the model's test-set accuracy / F1 and AIF360 group metrics (model-level,
    computed once) and the partition's Pruned accuracy / F1 on its simulation points."""

    COLS = ["Partition ID", "Original Accuracy", "Original F1 Score", "Pruned Accuracy", "Pruned F1", "DI", "SPD",
            "EOD", "AOD", "ERD", "CNT", "TI"]

    def __init__(self, out_dir: str, preset: Preset, mlp, seed: int, resume: bool):
        import csv

        from ..analysis.metrics import all_metrics
        from ..data import tabular

        ds = tabular.load(preset.suite, seed=seed, mlp=mlp)
        m = all_metrics(ds.X_test, ds.y_test, mlp.predict(ds.X_test), preset.resolved().pa_idx[0])
        self.model_vals = [m["accuracy"], m["f1"]]
        self.group_vals = [m[k] for k in ("DI", "SPD", "EOD", "AOD", "ERD", "CNT", "TI")]
        self.synthetic = bool(getattr(ds, "synthetic", False))
        family = mlp.name.split("-")[0]
        self.path = os.path.join(out_dir, f"synthetic-{preset.suite}-predicted-{family}-metrics.csv")
        os.makedirs(out_dir, exist_ok=True)
        exists = resume and os.path.exists(self.path)
        self.fp = open(self.path, "a" if exists else "w", newline="")
        self.wr = csv.writer(self.fp, dialect="excel")
        if not exists:
            self.wr.writerow(self.COLS)

    def write(self, positions: np.ndarray, recs) -> None:
        c = recs.cols
        for k, pos in enumerate(positions):
            self.wr.writerow([int(pos) + 1] + self.model_vals + [float(c["pruned_acc"][k]), float(c["pruned_f1"][k])]
                             + self.group_vals)
        self.fp.flush()

    def close(self) -> None:
        self.fp.close()


def run_preset(preset: Preset, models: Optional[List[str]] = None, weights: str = "zoo", out_dir: str = "results",
               cfg: Optional[VerifyConfig] = None, info: Optional[D.DistInfo] = None,
               max_partitions: Optional[int] = None, resume: bool = False, seed: int = 0,
               accuracy: bool = True, verbose: bool = True, escalate: int = 1,
               concurrency: int = 1, anytime_budget: Optional[float] = None,
               metrics_csv: Optional[bool] = None, balance: str = "queue", start_partition: int = 0) -> List[Dict]:
    """``escalate`` > 1: every round's UNKNOWN partitions are re-distributed over all ranks and
    retried with ``escalate`` x the node budget (residual work stealing).  ``concurrency`` > 1:
    each rank verifies that many chunks of a round at once, one host thread + HIP stream each
    (a round is then ``chunk x concurrency`` partitions per rank).  ``anytime_budget`` (seconds
    per model, e.g. the preset's hard timeout): every round gets the share of the model's
    remaining budget proportional to its partitions and spends it on deeper sound BaB passes and
    falsifier rounds over its UNKNOWN residue (VerifyConfig.anytime_seconds).  ``metrics_csv``
    (default: on for the fork's ``experiment/*`` presets): rank 0 also writes the per-partition
    ``synthetic-<dataset>-predicted-<family>-metrics.csv`` of the experiment drivers
    (src/AC/Verify-AC-experiment-new.py:482-542).  ``balance``: "queue" (several ranks: dynamic
    unit claiming from the store, see the module docstring) or "strided"."""
    info = info or D.DistInfo()
    if balance not in ("queue", "strided"):
        raise ValueError(f"balance must be 'queue' or 'strided', got {balance!r}")
    queue = balance == "queue" and info.world > 1
    claim = _claim_fn(info) if queue else None
    # per-invocation nonce of the unit-queue keys: every rank counts its own run_preset calls in the
    # store (SPMD: the same count on every rank), so a second call with the same preset / model /
    # seed gets fresh counters instead of an exhausted one
    run_id = claim(f"fairify/runs/{info.rank}") if queue else 0
    grid = preset.grid(seed=seed)
    q = preset.resolved()
    order = processing_order(grid, seed=seed)
    if start_partition:
        # a contiguous block of the seeded order (one part of a run split over calls / jobs; the parts
        # of a model partition its grid and their Table-V counts add up)
        order = order[int(start_partition):]
    total = len(order) if max_partitions is None else min(len(order), int(max_partitions))
    cfg = cfg or VerifyConfig(sim_size=preset.sim_size, soft_timeout=preset.soft_timeout,
                              hard_timeout=preset.hard_timeout, heuristic_p=preset.heuristic_p, seed=seed)
    n0 = q.n
    if metrics_csv is None:
        metrics_csv = preset.name.startswith("experiment/")
    if metrics_csv:
        cfg = replace(cfg, pruned_metrics=True)
    rows_out: List[Dict] = []
    streams = StreamPool(info.device, concurrency)
    pa_name = ",".join(a for a in preset.query.pa if preset.domain().has(a))
    for name in (models or list(preset.models)):
        mlp = get_model(name, weights=weights, seed=seed)
        be = Backend(mlp, device=info.device)
        heap.freeze()                # the model's setup objects: out of the cycle collector's scans
        acc, acc_src = model_accuracy(mlp, preset.suite, seed, with_source=True) if accuracy else (None, None)
        state_path = os.path.join(out_dir, "state", f"{name}.npz")
        csv_path = os.path.join(out_dir, f"{name}.csv")
        done = np.zeros(total, dtype=bool)            # checkpoint: finished processing positions
        if resume and os.path.exists(state_path):
            done = _load_done(state_path, total)
        todo = np.nonzero(~done)[0]
        mine = todo[info.rank::info.world]
        writer = PartitionCSV(csv_path, resume=resume) if info.is_main else None
        mwriter = _MetricsCSV(out_dir, preset, mlp, seed, resume) if (metrics_csv and info.is_main) else None
        # rank 0 formats/writes round r (native formatter, GIL released) and checkpoints it on a
        # background thread while round r+1's chunks drive the GPU; one worker keeps the order
        io = ThreadPoolExecutor(max_workers=1) if info.is_main else None
        pending = []
        wire_bytes = [0, 0]
        table_cols: Dict[str, List[np.ndarray]] = {k: [] for k in _TABLE_COLS}
        mask_parts: List[tuple] = []        # K6: (positions, grid ids, packed masks) per round
        timer = StageTimer(info.device)
        t0 = time.time()
        per_round = cfg.chunk * streams.workers
        rounds = int(np.ceil(len(todo) / max(1, per_round * info.world))) if len(todo) else 0
        stopped = False
        last_note = time.time()
        inflight = None      # (async gather handle, per-rank positions) of the previous round
        rank_work = [0.0, 0]  # this rank's BaB node expansions and partitions (balance report)
        rank_snodes = np.zeros(len(STAGE_NODE_COLS))   # ... of them per stage (pipeline.STAGE_NODE_COLS)

        def flush(item):
            handle, rpos, retried, expect = item
            bufs = handle.wait()
            if not info.is_main:
                return
            if rpos is None:        # unit queue: every rank's buffer carries its claimed positions
                split = [_unpack_positions(b) for b in bufs]
                rpos, bufs = [p for p, _ in split], [b for _, b in split]
                got = np.sort(np.concatenate(rpos)) if rpos else np.zeros(0, np.int64)
                if got.size != expect.size or not np.array_equal(got, np.sort(expect)):
                    raise RuntimeError(f"unit queue: ranks verified {got.size} positions of a round block of "
                                       f"{expect.size} (stale or shared queue key)")
            parts = [(p, wire.decode(b, order[p], acc, mlp.n_neurons, cfg.sim_size, q)) for p, b in zip(rpos, bufs)]
            gpos, grecs = wire.merge_rounds(parts)
            if grecs is None:
                return
            if retried is not None and retried[1] is not None:
                _replace(gpos, grecs, *retried)
            rows = pack(grecs, gpos, n0)
            cols = columns(rows, n0)
            if cfg.keep_masks and "mask_bits" in grecs.cols:
                mask_parts.append((gpos, grecs.cols["grid_id"], grecs.cols["mask_bits"]))
            if mwriter is not None:
                mwriter.write(gpos, grecs)
            for k in _TABLE_COLS:
                table_cols[k].append(cols[k])
            wire_bytes[0] += sum(len(b) for b in bufs)
            wire_bytes[1] += len(gpos)
            pending.append(io.submit(_write_round, writer, rows, n0, acc, done, state_path))
            if len(pending) > 2:
                pending.pop(0).result()

        for r in range(rounds):
            elapsed = D.all_reduce_max(info, time.time() - t0)
            if elapsed > cfg.hard_timeout:
                stopped = True
                break
            rblock = todo[r * per_round * info.world:(r + 1) * per_round * info.world]
            rpos = None if queue else _round_positions(todo, r, per_round, info.world)
            buf = wire.empty(q)
            codes = np.zeros(0, np.int8)
            rcfg = cfg
            if anytime_budget:
                # this round's share of the remaining per-model budget (all ranks agree: the
                # elapsed time is the global max and the round sizes are known everywhere)
                n_round = len(rblock)
                n_left = len(todo) - r * per_round * info.world
                share = max(0.0, (min(anytime_budget, cfg.hard_timeout) - elapsed) * n_round / max(1, n_left))
                rcfg = replace(cfg, anytime_seconds=0.9 * share)

            def run_ids(sp):
                return verify_chunk(be, mlp, q, grid, order[sp], rcfg, orig_acc=acc,
                                    time_budget=cfg.hard_timeout - elapsed, timer=timer)

            recs = None
            if queue:
                U = queue_unit_size(len(rblock), info.world, streams.workers, cfg.chunk)
                n_units = -(-len(rblock) // U)
                key = f"fairify/units/{run_id}/{preset.name}/{name}/{seed}/{r}"

                def worker(_):
                    done_units = []
                    while True:
                        u = claim(key)
                        if u >= n_units:
                            return done_units
                        sp = rblock[u * U:(u + 1) * U]
                        done_units.append((u, sp, run_ids(sp)))

                got = sorted((it for lst in streams.run(worker, [None] * streams.workers) for it in lst),
                             key=lambda it: it[0])
                pos = np.concatenate([sp for _, sp, _ in got]) if got else np.zeros(0, np.int64)
                if got:
                    recs = concat_records([rc for _, _, rc in got])
            else:
                pos = rpos[info.rank]
                if len(pos):
                    subs = [pos[s:s + cfg.chunk] for s in range(0, len(pos), cfg.chunk)]
                    recs = concat_records(streams.run(run_ids, subs))
            if recs is not None:
                buf = wire.encode(recs, q)
                codes = wire.verdict_codes(recs)
                rank_work[0] += float(recs.core["nodes"].sum())
                rank_work[1] += len(recs)
                if "stage_nodes" in recs.core:
                    rank_snodes += recs.core["stage_nodes"].sum(axis=0)
            retried = None
            if escalate > 1:
                all_codes = D.all_gather_int8(info, codes)
                all_pos = (D.all_gather_rows(info, np.asarray(pos, np.int64).reshape(-1, 1)).reshape(-1) if queue
                           else np.concatenate(rpos))
                retried = _residual_pass(be, mlp, q, grid, order, all_pos, all_codes, cfg, escalate,
                                         acc, info, timer, cfg.hard_timeout - elapsed)
            if queue:
                buf = _pack_positions(pos, buf)
            # this round's results travel to rank 0 while the next round computes
            handle = D.gather_bytes(info, buf, async_op=True)
            if inflight is not None:
                flush(inflight)
            inflight = (handle, rpos, retried, rblock)
            if faults.crash_after() >= 0:          # fault injection: crash only after a checkpoint
                flush(inflight)
                inflight = None
                for f in pending:
                    f.result()
                pending.clear()
            faults.maybe_crash(r + 1, info.rank)
            if verbose and info.is_main and time.time() - last_note > 20.0:
                last_note = time.time()
                print(f"[{preset.name}] {name}: round {r + 1}/{rounds}, "
                      f"{min(len(todo), (r + 1) * per_round * info.world)}/{len(todo)} partitions, "
                      f"{time.time() - t0:.0f}s", flush=True)
        if inflight is not None:
            flush(inflight)
        for f in pending:
            f.result()
        if io is not None:
            io.shutdown(wait=True)
        if mwriter is not None:
            mwriter.close()
        rank_busy = time.time() - t0
        wall = D.all_reduce_max(info, rank_busy)
        rank_nodes = D.all_gather_floats(info, rank_work[0])
        rank_parts = D.all_gather_floats(info, float(rank_work[1]))
        snodes = D.all_reduce_sum(info, rank_snodes)
        if info.is_main:
            tc = {k: (np.concatenate(v) if v else np.zeros(0)) for k, v in table_cols.items()}
            stage_codes = tc.pop("stage").astype(np.int64)
            row = table_v_row_columns(name, pa_name, grid_size=len(grid), wall=wall, **tc)
            row["stopped_by_hard_timeout"] = stopped
            row["original_acc"] = acc
            row["original_acc_source"] = acc_src
            # honest accounting: which stage decided (heuristic verdicts are the reference's
            # unsound retry; "milp" UNSAT rests on HiGHS's floating-point dual bound)
            v = tc["verdict"].astype(np.int64)
            row["sat_by_stage"] = {STAGES[k] or "none": int(((v == 1) & (stage_codes == k)).sum())
                                   for k in range(len(STAGES)) if ((v == 1) & (stage_codes == k)).any()}
            row["unsat_by_stage"] = {STAGES[k] or "none": int(((v == 2) & (stage_codes == k)).sum())
                                     for k in range(len(STAGES)) if ((v == 2) & (stage_codes == k)).any()}
            row["UNSAT_sound"] = int(((v == 2) & ~np.isin(stage_codes, [STAGES.index("heuristic"),
                                                                        STAGES.index("milp")])).sum())
            row["UNSAT_heuristic"] = int(((v == 2) & (stage_codes == STAGES.index("heuristic"))).sum())
            row["UNSAT_milp"] = int(((v == 2) & (stage_codes == STAGES.index("milp"))).sum())
            # MILP "unsat" claims left UNKNOWN (default: a floating-point dual bound is no proof)
            row["UNK_milp_unverified"] = int(((v == 0) & (stage_codes == STAGES.index("milp"))).sum())
            sound_sat = int(((v == 1) & (stage_codes != STAGES.index("heuristic"))).sum())
            row["Cov_sound%"] = round(100.0 * (sound_sat + row["UNSAT_sound"]) / max(1, len(grid)), 2)
            if anytime_budget:
                row["anytime_budget_s"] = float(anytime_budget)
            row["wire_bytes_per_partition"] = round(wire_bytes[0] / max(1, wire_bytes[1]), 2)
            row["balance"] = "queue" if queue else ("strided" if info.world > 1 else "none")
            row["rank_nodes"] = [int(v) for v in rank_nodes]
            row["rank_partitions"] = [int(v) for v in rank_parts]
            # where the work went: node expansions per stage (all ranks) and rank 0's stage timers
            # (host-thread wall seconds, summed over concurrent threads: a breakdown, not a wall time)
            row["stage_nodes"] = {c: int(snodes[i]) for i, c in enumerate(STAGE_NODE_COLS)}
            row["stage_s"] = {k: round(v, 3) for k, v in sorted(timer.t.items(), key=lambda kv: -kv[1])}
            if cfg.keep_masks and mask_parts:
                from ..report.masks import write_masks

                row["unique_masks"] = write_masks(os.path.join(out_dir, "masks", f"{name}.npz"), mask_parts,
                                                  mlp.n_neurons, resume=resume)
            rows_out.append(row)
            if verbose:
                print(f"[{preset.name}] {name}: {row['SAT']} sat / {row['UNSAT']} unsat / {row['UNK']} unknown "
                      f"of {row['#P']} (grid {len(grid)}, cov {row['Cov%']}%) in {wall:.2f}s "
                      f"= {row['partitions_per_s']} partitions/s", flush=True)
    streams.close()
    if info.is_main:
        write_summary(os.path.join(out_dir, "summary.json"), rows_out,
                      {"preset": preset.name, "weights": weights, "n_ranks": info.world, "seed": seed,
                       "config": asdict(cfg)})
        if verbose and rows_out:
            print(format_table(rows_out), flush=True)
    return rows_out
