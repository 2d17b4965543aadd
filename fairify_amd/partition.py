"""Input-space partition grid (never materialised).

Re-design of the reference partitioner ``utils/input_partition.py:17-76`` (``partition`` +
``partitioned_ranges``) and its capped variant ``:78-182`` (``partition_df`` +
``partitioned_ranges_df``).  The reference builds the Cartesian product of per-attribute
chunks as a Python list of dicts (3.29 M dicts for ``stress/AC``) and shuffles it unseeded.
Here a partition is an integer id; its box is computed on demand by a mixed-radix decode
(vectorised on host, and inside the HIP kernels on device), and the processing order is a
seeded bijective permutation so runs are reproducible and resumable.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .spec import Domain, ResolvedQuery


@dataclass
class AttrChunks:
    index: int                 # feature index in the domain
    lo: np.ndarray             # [C] chunk lows
    hi: np.ndarray             # [C] chunk highs

    @property
    def count(self) -> int:
        return int(self.lo.shape[0])


def _chunks_reference(lo: int, hi: int, p: int) -> Optional[Tuple[np.ndarray, np.ndarray]]:
    """``partition()`` semantics (utils/input_partition.py:17-46)."""
    size = hi - lo + 1
    if size <= p:
        return None
    lows = np.arange(lo, hi + 1, p, dtype=np.int64)
    highs = np.minimum(lows + p - 1, hi)
    return lows, highs


def _chunks_capped(lo: int, hi: int, p: int, quirks: bool) -> Optional[Tuple[np.ndarray, np.ndarray]]:
    """``partition_df()`` semantics (utils/input_partition.py:78-109).

    The reference uses ``size = hi - lo`` and ``while cur_low < high`` which silently drops the
    value ``hi`` whenever ``(hi - lo) % p == 0``; ``quirks=True`` reproduces that, otherwise the
    last chunk is closed at ``hi``.
    """
    if hi - lo <= p:
        return None
    lows = np.arange(lo, hi if quirks else hi + 1, p, dtype=np.int64)
    highs = np.minimum(lows + p - 1, hi)
    return lows, highs


class Grid:
    """Mixed-radix partition grid over a domain (optionally restricted to an id subset)."""

    def __init__(self, domain: Domain, attrs: List[AttrChunks], subset: Optional[np.ndarray] = None,
                 partition_size: int = 0):
        self.domain = domain
        self.attrs = attrs
        self.partition_size = partition_size
        self.base_lo = domain.lo()
        self.base_hi = domain.hi()
        self.radix = np.array([a.count for a in attrs], dtype=np.int64)
        self.full_size = int(np.prod(self.radix)) if attrs else 1
        self.subset = None if subset is None else np.asarray(subset, dtype=np.int64)

    # ------------------------------------------------------------------ constructors
    @classmethod
    def reference(cls, domain: Domain, partition_size: int, order: Optional[Sequence[str]] = None) -> "Grid":
        names = list(order) if order is not None else domain.names
        attrs = []
        for name in names:
            i = domain.index(name)
            f = domain.features[i]
            ch = _chunks_reference(f.lo, f.hi, partition_size)
            if ch is not None:
                attrs.append(AttrChunks(i, ch[0], ch[1]))
        return cls(domain, attrs, partition_size=partition_size)

    @classmethod
    def capped(cls, domain: Domain, partition_size: int, pa: Sequence[str], max_partitions: int = 100,
               seed: int = 0, quirks: bool = True) -> "Grid":
        """``partitioned_ranges_df`` (utils/input_partition.py:111-182): PA first, then other
        attributes while the product stays <= max_partitions; sample if still too many."""
        cand: Dict[str, AttrChunks] = {}
        for i, f in enumerate(domain.features):
            ch = _chunks_capped(f.lo, f.hi, partition_size, quirks)
            if ch is not None:
                cand[f.name] = AttrChunks(i, ch[0], ch[1])
        prio = [a for a in pa if a in cand]
        others = [a for a in cand if a not in prio]
        chosen, est = [], 1
        for a in prio:
            est *= cand[a].count
            chosen.append(cand[a])
        for a in others:
            if est * cand[a].count <= max_partitions:
                est *= cand[a].count
                chosen.append(cand[a])
        g = cls(domain, chosen, partition_size=partition_size)
        if g.full_size > max_partitions:
            rng = np.random.default_rng(seed)
            g.subset = np.sort(rng.choice(g.full_size, size=max_partitions, replace=False))
        return g

    # ------------------------------------------------------------------ size / ids
    def __len__(self) -> int:
        return int(self.subset.shape[0]) if self.subset is not None else self.full_size

    def ids(self) -> np.ndarray:
        return self.subset.copy() if self.subset is not None else np.arange(self.full_size, dtype=np.int64)

    def decode(self, ids: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """Partition ids (grid-linear, row-major over ``attrs``) -> boxes ``lo, hi`` [B, n] int64."""
        ids = np.asarray(ids, dtype=np.int64)
        B = ids.shape[0]
        lo = np.broadcast_to(self.base_lo, (B, self.domain.n)).copy()
        hi = np.broadcast_to(self.base_hi, (B, self.domain.n)).copy()
        rem = ids.copy()
        for a in reversed(self.attrs):
            c = rem % a.count
            rem //= a.count
            lo[:, a.index] = a.lo[c]
            hi[:, a.index] = a.hi[c]
        return lo, hi

    def encode(self, x: np.ndarray) -> np.ndarray:
        """Points [B, n] -> grid-linear partition id (-1 if outside the domain)."""
        x = np.asarray(x)
        B = x.shape[0]
        ids = np.zeros(B, dtype=np.int64)
        inside = np.all((x >= self.base_lo) & (x <= self.base_hi), axis=1)
        for a in self.attrs:
            c = np.searchsorted(a.lo, x[:, a.index], side="right") - 1
            c = np.clip(c, 0, a.count - 1)
            inside &= (x[:, a.index] >= a.lo[c]) & (x[:, a.index] <= a.hi[c])
            ids = ids * a.count + c
        ids[~inside] = -1
        return ids

    def box_dict(self, pid: int) -> Dict[str, List[int]]:
        lo, hi = self.decode(np.array([pid]))
        return {f.name: [int(lo[0, i]), int(hi[0, i])] for i, f in enumerate(self.domain.features)}

    def decode_desc(self) -> Dict[str, np.ndarray]:
        """Per-input-dim descriptor of the device decode (``fa_decode_kernel``, K1): the dim's
        mixed-radix radix (0 = not partitioned), the divisor (product of the radices of the
        attributes after it in row-major order), its slice of the chunk tables, the domain range."""
        n = self.domain.n
        radix = np.zeros(n, dtype=np.int32)
        div = np.ones(n, dtype=np.int64)
        off = np.zeros(n, dtype=np.int32)
        t = self.decode_table()
        later = 1
        for k in range(len(self.attrs) - 1, -1, -1):
            a = self.attrs[k]
            radix[a.index] = a.count
            div[a.index] = later
            off[a.index] = int(t["chunk_off"][k])
            later *= a.count
        return {"radix": radix, "div": div, "chunk_off": off,
                "base_lo": self.base_lo.astype(np.float32), "base_hi": self.base_hi.astype(np.float32),
                "chunk_lo": t["chunk_lo"].astype(np.float32), "chunk_hi": t["chunk_hi"].astype(np.float32)}

    def decode_table(self) -> Dict[str, np.ndarray]:
        """Flat arrays describing the grid for the device-side decode."""
        offs = np.zeros(len(self.attrs) + 1, dtype=np.int64)
        for k, a in enumerate(self.attrs):
            offs[k + 1] = offs[k] + a.count
        return {
            "attr_index": np.array([a.index for a in self.attrs], dtype=np.int32),
            "radix": self.radix.astype(np.int64),
            "chunk_off": offs,
            "chunk_lo": np.concatenate([a.lo for a in self.attrs]) if self.attrs else np.zeros(0, np.int64),
            "chunk_hi": np.concatenate([a.hi for a in self.attrs]) if self.attrs else np.zeros(0, np.int64),
            "base_lo": self.base_lo.copy(),
            "base_hi": self.base_hi.copy(),
        }


def reference_partition_list(range_dict: Dict[str, List[int]], partition_size: int) -> List[Dict[str, List[int]]]:
    """Materialised list of box dicts in the reference's product order (test oracle only)."""
    import itertools

    parts, keys = [], []
    for k, (lo, hi) in range_dict.items():
        ch = _chunks_reference(lo, hi, partition_size)
        if ch is not None:
            keys.append(k)
            parts.append([[int(a), int(b)] for a, b in zip(*ch)])
    out = []
    for comb in itertools.product(*parts):
        d = {k: list(v) for k, v in range_dict.items() if k not in keys}
        for k, c in zip(keys, comb):
            d[k] = c
        out.append(d)
    return out


# --------------------------------------------------------------------------------------
# Seeded bijective order (replaces the unseeded ``shuffle(p_list)``, src/AC/Verify-AC.py:74)
# --------------------------------------------------------------------------------------

_MASK64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix(x: np.ndarray, key: np.uint64) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (x ^ key) * np.uint64(0x9E3779B97F4A7C15)
        z ^= z >> np.uint64(29)
        z *= np.uint64(0xBF58476D1CE4E5B9)
        z ^= z >> np.uint64(32)
    return z


def permute(idx: np.ndarray, n: int, seed: int) -> np.ndarray:
    """Bijection of [0, n) (4-round Feistel on the next even power of two + cycle walking)."""
    idx = np.asarray(idx, dtype=np.uint64)
    if n <= 1:
        return idx.astype(np.int64)
    bits = max(2, int(np.ceil(np.log2(n))))
    bits += bits & 1
    half = bits // 2
    hmask = np.uint64((1 << half) - 1)
    keys = [np.uint64((seed * 0x632BE59BD9B4E019 + r * 0x85EBCA77C2B2AE63 + 1) & 0xFFFFFFFFFFFFFFFF)
            for r in range(4)]

    def once(v):
        left, right = v >> np.uint64(half), v & hmask
        for k in keys:
            left, right = right, left ^ (_mix(right, k) & hmask)
        return (left << np.uint64(half)) | right

    out = once(idx)
    bad = out >= np.uint64(n)
    while np.any(bad):
        out[bad] = once(out[bad])
        bad = out >= np.uint64(n)
    return out.astype(np.int64)


def processing_order(grid: Grid, seed: int, shuffle: bool = True) -> np.ndarray:
    """Partition ids in processing order (the seeded analogue of the reference shuffle)."""
    ids = grid.ids()
    if not shuffle:
        return ids
    return ids[permute(np.arange(len(ids)), len(ids), seed)]


def shard(order: np.ndarray, rank: int, world: int) -> np.ndarray:
    """Strided shard of the processing order (balanced: easy/hard partitions interleave)."""
    return order[rank::world]
