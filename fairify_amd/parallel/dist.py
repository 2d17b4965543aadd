"""Data-parallel execution over the partition grid (one process per GPU, RCCL over xGMI).

The reference has no parallelism at all (a single ``for model: for partition:`` loop,
src/AC/Verify-AC.py:78,109).  Here the seeded partition order is sharded across ranks
(strided, so easy and hard partitions interleave), every rank verifies its shard on its own
GPU, and the small per-partition results are exchanged with collectives:

* ``all_gather`` of int8 verdicts, fp32 stats rows and packed dead-neuron bitmasks (RCCL
  all-gather; the largest exchange — 3.29 M x 26 B masks for stress/AC — is chunked);
* ``all_reduce(MAX)`` of elapsed time for the global hard timeout / bench timing;
* ``all_reduce(SUM)`` of the SAT/UNSAT/UNK counters.

Backend ``nccl`` is RCCL on ROCm; CPU runs (tests) use ``gloo``.  Rendezvous is 127.0.0.1.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    initialized: bool = False

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init(device_type: Optional[str] = None) -> DistInfo:
    """Initialise from torchrun env vars (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*); no-op for 1 proc."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if device_type == "cuda":
        # one process per GPU; ranks beyond the visible devices (rehearsals with several ranks
        # on one GPU) share devices round-robin
        n_dev = max(1, torch.cuda.device_count())
        torch.cuda.set_device(local % n_dev)
        dev = torch.device("cuda", local % n_dev)
    else:
        dev = torch.device("cpu")
    info = DistInfo(rank=rank, world=world, local_rank=local, device=dev)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        backend = "nccl" if device_type == "cuda" else "gloo"
        # FAIRIFY_DIST_BACKEND=gloo: host collectives (e.g. several ranks sharing one GPU, where
        # RCCL refuses duplicate devices); the default on GPUs is nccl == RCCL over xGMI
        backend = os.environ.get("FAIRIFY_DIST_BACKEND", backend)
        if backend == "nccl":
            dist.init_process_group(backend, rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
        info.initialized = True
    elif dist.is_initialized():
        info.initialized = True
    return info


def barrier(info: DistInfo) -> None:
    if info.initialized:
        if _dev(info).type == "cuda":
            dist.barrier(device_ids=[info.device.index])
        else:
            dist.barrier()


def _dev(info: DistInfo) -> torch.device:
    """Device of collective buffers: the GPU for RCCL, the host for gloo."""
    if info.device.type == "cuda" and dist.is_initialized() and dist.get_backend() == "nccl":
        return info.device
    return torch.device("cpu")


def all_reduce_max(info: DistInfo, x: float) -> float:
    if not info.initialized:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_dev(info))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_sum(info: DistInfo, arr: np.ndarray) -> np.ndarray:
    if not info.initialized:
        return arr
    t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float64)).to(_dev(info))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def backend_name(info: DistInfo) -> str:
    """``nccl`` (RCCL on ROCm), ``gloo`` or ``none`` for a single process."""
    return dist.get_backend() if info.initialized and dist.is_initialized() else "none"


def all_gather_floats(info: DistInfo, x: float) -> List[float]:
    """One float per rank, in rank order (e.g. per-rank step times for the skew report)."""
    if not info.initialized:
        return [float(x)]
    t = torch.tensor([x], dtype=torch.float64, device=_dev(info))
    out = [torch.zeros_like(t) for _ in range(info.world)]
    dist.all_gather(out, t)
    return [float(v.item()) for v in out]


def all_gather_rows(info: DistInfo, arr: np.ndarray, chunk_bytes: int = 64 << 20) -> np.ndarray:
    """Gather variable-length row blocks [n_i, ...] from every rank -> concatenated in rank order.

    Sizes are exchanged first; payloads are padded to the max and gathered in chunks of
    ``chunk_bytes`` per rank (large mask tables stay within RCCL-friendly message sizes).
    """
    if not info.initialized:
        return arr
    dev = _dev(info)
    arr = np.ascontiguousarray(arr)
    n = torch.tensor([arr.shape[0]], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(info.world)]
    dist.all_gather(ns, n)
    ns = [int(v.item()) for v in ns]
    nmax = max(ns)
    row_shape = arr.shape[1:]
    raw = arr.view(np.uint8).reshape(arr.shape[0], -1) if arr.size else np.zeros((arr.shape[0], int(np.prod(row_shape)) * arr.dtype.itemsize), np.uint8)
    rb = raw.shape[1]
    pad = np.zeros((nmax, rb), dtype=np.uint8)
    pad[:arr.shape[0]] = raw
    out = np.zeros((info.world, nmax, rb), dtype=np.uint8)
    rows_per = max(1, chunk_bytes // max(1, rb))
    for s in range(0, max(nmax, 1), rows_per):
        e = min(nmax, s + rows_per)
        if e <= s:
            break
        src = torch.from_numpy(pad[s:e].copy()).to(dev)
        bufs = [torch.empty_like(src) for _ in range(info.world)]
        dist.all_gather(bufs, src)
        for r in range(info.world):
            out[r, s:e] = bufs[r].cpu().numpy()
    parts = [out[r, :ns[r]].copy().view(arr.dtype).reshape((ns[r],) + row_shape) for r in range(info.world)]
    return np.concatenate(parts, axis=0) if parts else arr


def broadcast_array(info: DistInfo, arr: Optional[np.ndarray], src: int = 0) -> np.ndarray:
    """Broadcast a numpy array (e.g. model weights / query spec) from ``src``."""
    if not info.initialized:
        return arr
    objs = [arr if info.rank == src else None]
    dist.broadcast_object_list(objs, src=src)
    return objs[0]


def pack_bits(mask: np.ndarray) -> np.ndarray:
    """[P, N] bool -> [P, ceil(N/8)] uint8 (dead-neuron bitmasks for the gather)."""
    return np.packbits(mask.astype(bool), axis=1)


def unpack_bits(bits: np.ndarray, n: int) -> np.ndarray:
    return np.unpackbits(bits, axis=1)[:, :n].astype(bool)


def destroy(info: DistInfo) -> None:
    if info.initialized and dist.is_initialized():
        dist.destroy_process_group()
