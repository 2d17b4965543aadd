"""Cross-rank load balancing of (model, chunk) work units and node-level host resources.

Strong-scaling bench step (bench.py): the seeded partition order of every model is cut into
contiguous units of ``unit_size`` partitions; every unit is verified by exactly one rank, so a
step's verdict totals do not depend on the assignment (per-partition verdicts are independent
of which partitions share a chunk: tests/test_determinism_gpu.py, tests/test_bench_launch.py).
The first step assigns units by a size prior; afterwards every rank reports the cost of the
units it ran (BaB node expansions weighted by the model's multiply-adds, plus a fixed cost per
partition), the costs are summed over ranks (one ``all_reduce``, RCCL), and the next step
uses a deterministic LPT schedule (longest unit first onto the least loaded rank, ties to the
lower rank / unit index) -- SURVEY §2.4.2 "work stealing" / §7.5 "heavy-tailed work", with the
balancing decided once per step instead of by messages between ranks.  The reference is
sequential (src/AC/Verify-AC.py:78,109).

Host resources: one 8-GPU node runs 8 ranks, each with its own host threads / HIP streams and
MILP pool.  ``gpu_local_cpus`` reads which CPUs are local to rank r's GPU from sysfs (KFD topology
-> PCI address -> ``local_cpulist``; no HIP call, so it runs before the GPU is touched);
``rank_cpuset`` splits each GPU-local CPU set evenly among the ranks whose GPUs share it (the
ranks of one socket), falling back to the r-th contiguous slice of the allowed CPUs when sysfs
gives nothing usable; ``pin_rank`` applies it before any GPU call, ``host_threads`` sizes the
pools from that slice.
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
def parse_cpulist(text: str) -> List[int]:
    """sysfs cpulist ("0-31,64-95") -> sorted CPU ids."""
    out = set()
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    return sorted(out)


def _visible(n: int) -> List[int]:
    """KFD GPU indices this process sees, in device order (ROCR_VISIBLE_DEVICES, then
    HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES; integer lists only -- anything else: all)."""
    idx = list(range(n))
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is None or v.strip() == "":
            continue
        try:
            sel = [int(t) for t in v.split(",") if t.strip() != ""]
        except ValueError:
            return idx
        idx = [idx[k] for k in sel if 0 <= k < len(idx)]
    return idx


def gpu_pci_addresses(sysfs: str = "/sys", visible_only: bool = True) -> List[str]:
    """PCI addresses ("dddd:bb:dd.f") of the GPUs in KFD topology order (the order ROCr
    enumerates them), restricted to the visible devices (``visible_only``; else every GPU of
    the node, indexed by physical id).  [] when the topology is unreadable."""
    base = os.path.join(sysfs, "class", "kfd", "kfd", "topology", "nodes")
    try:
        nodes = sorted((int(d) for d in os.listdir(base) if d.isdigit()))
    except OSError:
        return []
    addrs = []
    for nd in nodes:
        try:
            with open(os.path.join(base, str(nd), "properties")) as f:
                props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0")) <= 0:        # CPU node
            continue
        loc, dom = int(props.get("location_id", "0")), int(props.get("domain", "0"))
        addrs.append(f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 0x7}")
    return [addrs[k] for k in _visible(len(addrs))] if visible_only else addrs


def gpu_local_cpus(device_index: int, sysfs: str = "/sys", visible_only: bool = True) -> List[int]:
    """CPUs local to GPU ``device_index`` (its PCI device's ``local_cpulist``); [] if unknown."""
    addrs = gpu_pci_addresses(sysfs, visible_only)
    if not addrs:
        return []
    addr = addrs[device_index % len(addrs)]
    try:
        with open(os.path.join(sysfs, "bus", "pci", "devices", addr, "local_cpulist")) as f:
            return parse_cpulist(f.read())
    except (OSError, ValueError):
        return []


def _slice(cpus: Sequence[int], k: int, n: int) -> List[int]:
    cpus = sorted(cpus)
    m = len(cpus)
    if n <= 1 or m == 0:
        return list(cpus)
    if m < n:
        return [cpus[k % m]]
    return list(cpus[(k * m) // n:((k + 1) * m) // n])


def rank_cpuset(local_rank: int, local_world: int, cpus: Sequence[int] = None, sysfs: str = "/sys",
                numa: bool = True) -> List[int]:
    """This rank's CPUs: with ``numa``, the CPUs local to its GPU (sysfs), split evenly among the
    ranks of this node whose GPUs report the same local set; otherwise (or when sysfs gives no
    usable set) the local_rank-th of local_world contiguous slices of ``cpus`` (default: this
    process's affinity set).  At least one CPU each."""
    cpus = sorted(os.sched_getaffinity(0)) if cpus is None else sorted(cpus)
    if local_world <= 1 or not cpus:
        return list(cpus)
    if numa:
        allowed = set(cpus)
        # a launcher that gives each rank only its own GPU (HIP / ROCR_VISIBLE_DEVICES = one id)
        # leaves fewer visible GPUs than local ranks: then local rank r is physical GPU r of the
        # node's KFD topology (an index into the visible list would make every rank a peer of all
        # the others); with fewer GPUs than ranks even there, the peers are unknown -> slices
        vis = len(gpu_pci_addresses(sysfs)) >= local_world
        if not vis and len(gpu_pci_addresses(sysfs, visible_only=False)) < local_world:
            return _slice(cpus, local_rank, local_world)
        sets = [tuple(c for c in gpu_local_cpus(r, sysfs, visible_only=vis) if c in allowed)
                for r in range(local_world)]
        if all(sets):
            peers = [r for r in range(local_world) if sets[r] == sets[local_rank]]
            return _slice(sets[local_rank], peers.index(local_rank), len(peers))
    return _slice(cpus, local_rank, local_world)


def pin_rank(local_rank: int, local_world: int) -> List[int]:
    """Restrict this process (and the threads it starts afterwards) to its CPUs (GPU-local when
    sysfs tells, ``rank_cpuset``).  Call before importing torch / touching the GPU.
    FAIRIFY_NO_PIN=1 disables it, FAIRIFY_PIN_NUMA=0 uses plain contiguous slices."""
    if os.environ.get("FAIRIFY_NO_PIN") == "1" or local_world <= 1 or not hasattr(os, "sched_setaffinity"):
        return sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else []
    mine = rank_cpuset(local_rank, local_world, numa=os.environ.get("FAIRIFY_PIN_NUMA", "1") != "0")
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
