"""K1 partition decode: the device kernel (fa_decode_kernel) vs the host mixed-radix decode, and
the descriptor it is driven by (CPU)."""
import numpy as np
import pytest
import torch

from fairify_amd import presets
from fairify_amd.partition import Grid, processing_order

PRESETS = ["src/AC-sex", "stress/BM", "src/GC-age", "relaxed/AC", "targeted/AC", "experiment/AC-3"]


def _desc_decode(grid: Grid, ids: np.ndarray):
    """The kernel's per-dim arithmetic on the host: (id // div) % radix -> chunk table slice."""
    d = grid.decode_desc()
    n0 = d["radix"].shape[0]
    lo = np.broadcast_to(d["base_lo"], (ids.size, n0)).copy()
    hi = np.broadcast_to(d["base_hi"], (ids.size, n0)).copy()
    for k in range(n0):
        if d["radix"][k]:
            c = (ids // d["div"][k]) % d["radix"][k]
            lo[:, k] = d["chunk_lo"][d["chunk_off"][k] + c]
            hi[:, k] = d["chunk_hi"][d["chunk_off"][k] + c]
    return lo, hi


@pytest.mark.parametrize("name", PRESETS)
def test_decode_desc_matches_host_decode(name):
    grid = presets.get(name).grid()
    order = processing_order(grid, seed=3)
    ids = order[:: max(1, len(order) // 5000)]
    lo, hi = grid.decode(ids)
    dlo, dhi = _desc_decode(grid, ids)
    assert np.array_equal(dlo, lo.astype(np.float32))
    assert np.array_equal(dhi, hi.astype(np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("name", PRESETS)
def test_decode_kernel_matches_host(cuda, name):
    from fairify_amd.ops import hip as H

    grid = presets.get(name).grid()
    order = processing_order(grid, seed=1)
    for ids in (order[:4099], order[-37:], order[:0]):
        lo, hi = H.decode(grid, torch.from_numpy(np.ascontiguousarray(ids)).to(cuda))
        hlo, hhi = grid.decode(ids)
        assert torch.equal(lo.cpu(), torch.from_numpy(hlo.astype(np.float32)))
        assert torch.equal(hi.cpu(), torch.from_numpy(hhi.astype(np.float32)))


@pytest.mark.gpu
def test_trace_marker_kernel_runs(cuda):
    from fairify_amd.ops import hip as H

    H.trace_marker(cuda, 1)
    torch.cuda.synchronize(cuda)
