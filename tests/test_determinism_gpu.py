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
