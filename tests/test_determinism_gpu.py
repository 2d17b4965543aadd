"""Race / determinism checks on the GPU (no GPU sanitizer on this pool, so data
races in LDS staging, wave-private slabs and the BaB node pool are caught as run-to-run or
serial-vs-concurrent differences).

* the register-resident kernels are bitwise reproducible launch to launch;
* a chunk verified on 4 host threads / HIP streams concurrently (one BaB runtime per thread)
  gives exactly the verdicts and counterexamples of the serial run.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

from fairify_amd import presets
from fairify_amd.engine.pipeline import VerifyConfig, verify_chunk
from fairify_amd.models.mlp import random_mlp
from fairify_amd.models.zoo import get_model
from fairify_amd.ops.backend import Backend
from fairify_amd.partition import processing_order

pytestmark = pytest.mark.gpu


def test_bound_kernels_bitwise_reproducible(cuda):
    m = random_mlp(13, [100, 100], seed=1, bias_scale=0.3)
    be = Backend(m, cuda)
    g = torch.Generator().manual_seed(0)
    lo = torch.randint(0, 20, (4096, 13), generator=g).float()
    hi = lo + torch.randint(0, 5, (4096, 13), generator=g).float()
    hi[:, 8] = lo[:, 8]
    lo, hi = lo.to(cuda), hi.to(cuda)
    a = be.bounds(lo, hi, mode="symbolic", fold=(8,))
    b = be.bounds(lo, hi, mode="symbolic", fold=(8,))
    for x, y in ((a.out_lb, b.out_lb), (a.out_ub, b.out_ub), (a.Lc, b.Lc), (a.U0, b.U0)):
        assert torch.equal(x, y)
    p1 = be.point_bounds(lo)
    p2 = be.point_bounds(lo)
    assert torch.equal(p1[0], p2[0]) and torch.equal(p1[1], p2[1])


def test_concurrent_streams_match_serial(cuda):
    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    order = processing_order(grid, 0)
    chunks = [order[i * 512:(i + 1) * 512] for i in range(4)]
    m = get_model("AC-5", weights="random", seed=0)
    be = Backend(m, cuda)
    cfg = VerifyConfig(sim_size=256, node_budget=512, smt_backend="none")
    serial = [verify_chunk(be, m, q, grid, ids, cfg) for ids in chunks]

    def run(ids):
        s = torch.cuda.Stream(cuda)
        with torch.cuda.stream(s):
            out = verify_chunk(be, m, q, grid, ids, cfg)
            torch.cuda.current_stream(cuda).synchronize()
        return out

    with ThreadPoolExecutor(4) as ex:
        conc = list(ex.map(run, chunks))
    for a, b in zip(serial, conc):
        assert [r["verdict"] for r in a] == [r["verdict"] for r in b]
        for ra, rb in zip(a, b):
            if ra["verdict"] == "sat":
                assert np.array_equal(ra["c1"], rb["c1"]) and np.array_equal(ra["c2"], rb["c2"])


@pytest.mark.parametrize("hidden", [[5, 5], [5] * 9, [3, 3, 3, 3], [8, 4, 8], [16, 8]])
def test_symbolic_bounds_independent_of_row_position(cuda, hidden):
    """A box's bounds must not depend on which rows share its wave / MFMA tile (the packed
    narrow-network kernel puts several boxes in one tile, and BaB node order follows device
    atomics): a permuted batch gives bitwise the same bounds per box."""
    m = random_mlp(13, hidden, seed=len(hidden), bias_scale=0.3)
    be = Backend(m, cuda)
    g = torch.Generator().manual_seed(1)
    R = 1003
    lo = torch.randint(0, 20, (R, 13), generator=g).float()
    hi = lo + torch.randint(0, 5, (R, 13), generator=g).float()
    hi[:, 8] = lo[:, 8]
    perm = torch.randperm(R, generator=g)
    a = be.bounds(lo.to(cuda), hi.to(cuda), mode="symbolic", fold=(8,), keep_layers=True)
    b = be.bounds(lo[perm].to(cuda), hi[perm].to(cuda), mode="symbolic", fold=(8,), keep_layers=True)
    inv = torch.argsort(perm).to(cuda)
    for x, y in ((a.out_lb, b.out_lb), (a.out_ub, b.out_ub), (a.Lc, b.Lc), (a.Uc, b.Uc), (a.L0, b.L0),
                 (a.Ue, b.Ue)):
        assert torch.equal(x, y[inv])
    for x, y in zip(a.layer_ub, b.layer_ub):
        assert torch.equal(x, y[inv])


def test_bab_verdicts_independent_of_chunk_composition(cuda):
    """The same partitions verified in one chunk and split over two chunks (different node pools,
    other partitions' nodes interleaved) give identical verdicts and counterexamples."""
    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    ids = processing_order(grid, 0)[:1024]
    cfg = VerifyConfig(sim_size=256, node_budget=512, escalate_budget=4096, escalate_max_open=256,
                       smt_backend="none")
    for name in ("AC-12", "AC-8", "AC-9"):
        m = get_model(name, weights="random", seed=0)
        be = Backend(m, cuda)
        whole = verify_chunk(be, m, q, grid, ids, cfg)
        parts = [verify_chunk(be, m, q, grid, ids[k::2], cfg) for k in range(2)]
        v = np.empty(len(ids), dtype=object)
        v[0::2], v[1::2] = parts[0].cols["verdict"], parts[1].cols["verdict"]
        assert list(v) == list(whole.cols["verdict"]), name
