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
    # FAIRIFY_DIST_INIT=1: form the process group even for a single rank (exercises the RCCL
    # communicator and collectives on a one-GPU box, where RCCL refuses two ranks per device)
    force = os.environ.get("FAIRIFY_DIST_INIT") == "1"
    if (world > 1 or force) and not dist.is_initialized():
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


class _Pending:
    """An in-flight :func:`gather_bytes`: ``wait()`` -> list of per-rank buffers on ``dst``
    (``None`` elsewhere)."""

    def __init__(self, work, bufs, sizes, is_dst, value=None):
        self.work, self.bufs, self.sizes, self.is_dst, self.value = work, bufs, sizes, is_dst, value

    def wait(self) -> Optional[List[np.ndarray]]:
        if self.value is not None or self.work is None:
            return self.value
        self.work.wait()
        self.work = None
        if not self.is_dst:
            return None
        self.value = [b[:n].cpu().numpy() for b, n in zip(self.bufs, self.sizes)]
        return self.value


def gather_bytes(info: DistInfo, buf: np.ndarray, dst: int = 0, async_op: bool = False):
    """Gather one variable-length uint8 buffer per rank to ``dst`` only (not an all-gather: the
    other ranks never need the results).  Sizes travel first (one int64 all-gather), payloads
    are padded to the largest.  ``async_op=True`` returns a handle whose ``wait()`` yields the
    list: the gather runs on the communicator's own stream (RCCL) / thread (gloo) while the
    caller's next round computes."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8).reshape(-1)
    if not info.initialized:
        p = _Pending(None, None, None, True, [buf])
        return p if async_op else p.wait()
    dev = _dev(info)
    n = torch.tensor([buf.size], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(info.world)]
    dist.all_gather(ns, n)
    sizes = [int(v.item()) for v in ns]
    nmax = max(1, max(sizes))
    src = torch.zeros(nmax, dtype=torch.uint8)
    src[:buf.size] = torch.from_numpy(buf)
    src = src.to(dev)
    is_dst = info.rank == dst
    bufs = [torch.empty(nmax, dtype=torch.uint8, device=dev) for _ in range(info.world)] if is_dst else None
    work = dist.gather(src, gather_list=bufs, dst=dst, async_op=True)
    p = _Pending(work, bufs, sizes, is_dst)
    p.src = src                     # keep the send buffer alive until the gather completes
    return p if async_op else p.wait()


def all_gather_int8(info: DistInfo, arr: np.ndarray) -> np.ndarray:
    """Variable-length int8 vectors (e.g. verdict codes) from every rank, concatenated in rank
    order on every rank."""
    arr = np.ascontiguousarray(arr, dtype=np.int8)
    if not info.initialized:
        return arr
    return all_gather_rows(info, arr.reshape(-1, 1)).reshape(-1)


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
