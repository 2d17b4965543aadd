"""Dead-neuron mask store: dedup + compaction of pruned subnetworks (K6).

The reference prunes one network per partition with ``np.delete`` per dead neuron
(``prune_neurons``, utils/prune.py:950-977) and derives the compression columns from the mask
(``compression_ratio``, :194-203).  Many partitions of a grid share the same mask, so here:

* every partition's final mask travels to rank 0 as a packed bitset (``fa_pack_masks_kernel``,
  ceil(N/8) B, numpy.packbits order; ``parallel/wire.py``);
* rank 0 stores ``masks/<model>.npz``: the unique masks (``np.unique`` over the packed rows),
  and per partition its processing position, grid id and index into the unique table;
* :func:`unique_subnets` compacts each UNIQUE mask's weight matrices once (``MLP.prune``) --
  the pruned networks the host solver / ``export-smt`` need, one per distinct mask instead of one
  per partition.
"""
from __future__ import annotations

import os
from typing import Dict, List, Sequence, Tuple

import numpy as np


def write_masks(path: str, parts: Sequence[Tuple[np.ndarray, np.ndarray, np.ndarray]], n_neurons: int,
                resume: bool = False) -> int:
    """``parts``: (positions, grid ids, packed masks) blocks -> deduplicated store at ``path``;
    with ``resume`` the rows of an existing store are kept (newer rows win per position).
    Returns the number of unique masks."""
    pos = np.concatenate([np.asarray(p, np.int64) for p, _, _ in parts])
    gid = np.concatenate([np.asarray(g, np.int64) for _, g, _ in parts])
    bits = np.concatenate([np.asarray(b, np.uint8) for _, _, b in parts])
    if resume and os.path.exists(path):
        old = load(path)
        keep = ~np.isin(old["position"], pos)
        pos = np.concatenate([old["position"][keep], pos])
        gid = np.concatenate([old["grid_id"][keep], gid])
        bits = np.concatenate([old["bits"][keep], bits])
    o = np.argsort(pos, kind="stable")
    pos, gid, bits = pos[o], gid[o], bits[o]
    uniq, inv = np.unique(bits, axis=0, return_inverse=True)
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = path + ".tmp.npz"
    np.savez_compressed(tmp, position=pos, grid_id=gid, mask_index=inv.reshape(-1).astype(np.int32),
                        unique_bits=uniq, n_neurons=np.int64(n_neurons))
    os.replace(tmp, path)
    return int(uniq.shape[0])


def load(path: str) -> Dict[str, np.ndarray]:
    """Store -> dict(position, grid_id, bits [P, ceil(N/8)], unique_bits, mask_index, n_neurons)."""
    z = np.load(path)    # plain arrays only (allow_pickle stays False)
    out = {k: z[k] for k in z.files}
    out["bits"] = out["unique_bits"][out["mask_index"]]
    return out


def unpack(bits: np.ndarray, n_neurons: int) -> np.ndarray:
    """Packed rows -> bool [rows, n_neurons]."""
    return np.unpackbits(np.asarray(bits, np.uint8), axis=1, count=n_neurons).astype(bool)


def layer_split(mask_row: np.ndarray, widths: Sequence[int]) -> List[np.ndarray]:
    out, o = [], 0
    for w in widths:
        out.append(mask_row[o:o + w])
        o += w
    return out


def unique_subnets(mlp, path: str):
    """(pruned MLP per unique mask, mask index per partition, grid ids): each distinct mask's
    network is compacted once (dead rows / columns deleted, ``MLP.prune``)."""
    st = load(path)
    if int(st["n_neurons"]) != mlp.n_neurons:
        raise ValueError(f"mask store has {int(st['n_neurons'])} neurons, model {mlp.name} has {mlp.n_neurons}")
    dense = unpack(st["unique_bits"], mlp.n_neurons)
    nets = [mlp.prune(layer_split(row, mlp.widths)) for row in dense]
    return nets, st["mask_index"], st["grid_id"]
