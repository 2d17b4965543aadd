"""Fault-injection knobs for failure-path tests (the reference has none).

All knobs are environment variables so they reach every rank of a torchrun job unchanged:

* ``FAIRIFY_FAULT_CRASH_AFTER=N``   — the runner raises :class:`InjectedFault` after it has
  checkpointed N rounds (simulates a rank/node failure mid-run; ``--resume`` must finish
  the job with results identical to an uninterrupted run);
* ``FAIRIFY_FAULT_CRASH_RANK=r``    — restrict the crash to rank r (default: every rank);
* ``FAIRIFY_FAULT_FORCE_UNKNOWN=p`` — turn a deterministic pseudo-random fraction p of the
  decided partitions of every chunk into UNKNOWN (simulates solver timeouts, exercising the
  heuristic retry / residual re-distribution paths);
* ``FAIRIFY_FAULT_SEED=s``          — seed of the forced-UNKNOWN selection.
"""
from __future__ import annotations

import os

import numpy as np


class InjectedFault(RuntimeError):
    pass


def _env_float(name: str, default: float = 0.0) -> float:
    v = os.environ.get(name)
    return float(v) if v not in (None, "") else default


def crash_after() -> int:
    v = os.environ.get("FAIRIFY_FAULT_CRASH_AFTER")
    return int(v) if v not in (None, "") else -1


def maybe_crash(rounds_done: int, rank: int) -> None:
    n = crash_after()
    if n < 0 or rounds_done < n:
        return
    r = os.environ.get("FAIRIFY_FAULT_CRASH_RANK")
    if r not in (None, "") and int(r) != rank:
        return
    raise InjectedFault(f"injected failure on rank {rank} after {rounds_done} checkpointed rounds")


def forced_unknown(grid_ids: np.ndarray) -> np.ndarray:
    """Boolean mask of partitions whose verdict is forced to UNKNOWN (deterministic in the id)."""
    p = _env_float("FAIRIFY_FAULT_FORCE_UNKNOWN")
    if p <= 0:
        return np.zeros(len(grid_ids), dtype=bool)
    seed = int(_env_float("FAIRIFY_FAULT_SEED", 0))
    h = (np.asarray(grid_ids, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(seed)) >> np.uint64(40)
    return (h.astype(np.float64) / float(1 << 24)) < p
