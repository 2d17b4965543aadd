"""Cross-rank load balancing of (model, chunk) work units and node-level host resources.

Strong-scaling bench step (bench.py): the seeded partition order of every model is cut into
contiguous units of ``unit_size`` partitions; every unit is verified by exactly one rank, so a
step's verdict totals do not depend on the assignment (per-partition verdicts are independent
of which partitions share a chunk: tests/test_determinism_gpu.py, tests/test_bench_launch.py).
The first step assigns units by a size prior; afterwards every rank reports the wall time of
the units it ran, the costs are summed over ranks (one ``all_reduce``, RCCL), and the next step
uses a deterministic LPT schedule (longest unit first onto the least loaded rank, ties to the
lower rank / unit index) -- SURVEY §2.4.2 "work stealing" / §7.5 "heavy-tailed work", with the
balancing decided once per step instead of by messages between ranks.  The reference is
sequential (src/AC/Verify-AC.py:78,109).

Host resources: one 8-GPU node runs 8 ranks, each with its own host threads / HIP streams and
MILP pool; ``rank_cpuset`` gives rank r of a node the r-th contiguous slice of the CPUs the
launcher may use, ``pin_rank`` applies it before any GPU call, ``host_threads`` sizes the pools
from that slice.
"""
from __future__ import annotations

import os
from typing import Dict, List, Sequence, Tuple

import numpy as np

Unit = Tuple[int, int]          # (model index, unit index within the model)


def make_units(n_models: int, n_parts: int, unit_size: int) -> List[Unit]:
    per = (n_parts + unit_size - 1) // max(1, unit_size)
    return [(k, j) for k in range(n_models) for j in range(per)]


def unit_ids(order: np.ndarray, j: int, unit_size: int) -> np.ndarray:
    return order[j * unit_size:(j + 1) * unit_size]


def lpt_assign(costs: Sequence[float], world: int) -> List[List[int]]:
    """Deterministic LPT: units in decreasing cost (ties: lower index first) onto the least
    loaded rank (ties: lower rank).  Returns the unit indices of every rank, in that order."""
    costs = np.asarray(costs, dtype=np.float64)
    order = sorted(range(len(costs)), key=lambda u: (-costs[u], u))
    load = np.zeros(world)
    out: List[List[int]] = [[] for _ in range(world)]
    for u in order:
        r = int(np.argmin(load))          # argmin returns the first (lowest) rank on ties
        out[r].append(u)
        load[r] += costs[u]
    return out


def rank_loads(assign: List[List[int]], costs: Sequence[float]) -> np.ndarray:
    c = np.asarray(costs, dtype=np.float64)
    return np.array([c[a].sum() if a else 0.0 for a in assign])


def prior_costs(units: Sequence[Unit], model_weight: Sequence[float], sizes: Dict[Unit, int]) -> np.ndarray:
    """Cost prior before any measurement: partitions x the model's weight (e.g. its neuron count)."""
    return np.array([float(sizes[u]) * float(model_weight[u[0]]) for u in units])


# ----------------------------------------------------------------------------------- host CPUs
def rank_cpuset(local_rank: int, local_world: int, cpus: Sequence[int] = None) -> List[int]:
    """The local_rank-th of local_world contiguous slices of ``cpus`` (default: this process's
    affinity set), at least one CPU each."""
    cpus = sorted(os.sched_getaffinity(0)) if cpus is None else sorted(cpus)
    n = len(cpus)
    if local_world <= 1 or n == 0:
        return list(cpus)
    if n < local_world:
        return [cpus[local_rank % n]]
    lo = (local_rank * n) // local_world
    hi = ((local_rank + 1) * n) // local_world
    return list(cpus[lo:hi])


def pin_rank(local_rank: int, local_world: int) -> List[int]:
    """Restrict this process (and the threads it starts afterwards) to its node slice of CPUs.
    Call before importing torch / touching the GPU.  FAIRIFY_NO_PIN=1 disables it."""
    if os.environ.get("FAIRIFY_NO_PIN") == "1" or local_world <= 1 or not hasattr(os, "sched_setaffinity"):
        return sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else []
    mine = rank_cpuset(local_rank, local_world)
    try:
        os.sched_setaffinity(0, set(mine))
    except OSError:
        return sorted(os.sched_getaffinity(0))
    return mine


def host_threads(cap: int = 8, floor: int = 1) -> int:
    """Host threads / HIP streams for this rank: the CPUs it may use, at most ``cap``."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(floor, min(cap, n))
