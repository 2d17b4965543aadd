"""Chunks whose partitions split the protected attribute's range differently (a PA wider than the
partition size, e.g. Adult age with P=10 -- the reference splits PA columns too,
utils/input_partition.py:48-76) are verified group by group and come back in input order."""
from dataclasses import replace

import numpy as np

from fairify_amd import presets
from fairify_amd.engine import exact
from fairify_amd.engine.pipeline import VerifyConfig, verify_chunk
from fairify_amd.models.zoo import get_model
from fairify_amd.ops.backend import Backend
from fairify_amd.partition import processing_order
from fairify_amd.spec import Query


def test_mixed_pa_ranges_in_one_chunk():
    pre = replace(presets.get("src/AC-sex"), query=Query(("age",)), partition_size=30)
    grid, q = pre.grid(), pre.resolved()
    ids = processing_order(grid, 0)[:40]
    lo, hi = grid.decode(ids)
    pa = q.pa_idx[0]
    assert len(np.unique(lo[:, pa])) > 1            # several PA ranges in the chunk
    m = get_model("AC-8", weights="random", seed=1)
    be = Backend(m)
    cfg = VerifyConfig(sim_size=128, node_budget=64, heuristic=False, residual_samples=0, smt_backend="none")
    recs = verify_chunk(be, m, q, grid, ids, cfg)
    assert list(recs.cols["grid_id"]) == list(ids)
    # same verdicts as verifying each PA group on its own
    for v in np.unique(lo[:, pa]):
        sel = np.nonzero(lo[:, pa] == v)[0]
        sub = verify_chunk(be, m, q, grid, ids[sel], cfg)
        assert list(sub.cols["verdict"]) == list(recs.cols["verdict"][sel])
    sat = np.nonzero(recs.cols["verdict"] == "sat")[0]
    assert sat.size
    X, XP = recs.cols["cex_x"][sat], recs.cols["cex_xp"][sat]
    assert exact.check_pair_constraints(X, XP, lo[sat], hi[sat], q.pa_idx, q.ra_idx, q.tau).all()
    assert exact.is_violation(m, X, XP).all()


def test_bab_solver_groups_pa_ranges_itself():
    """BaBSolver.solve splits a mixed-PA chunk into PA groups internally (no caller grouping
    needed): same verdicts as one solve per group, in input order."""
    from fairify_amd.engine.bab import BaBConfig, BaBSolver, pa_groups

    pre = replace(presets.get("src/AC-sex"), query=Query(("age",)), partition_size=30)
    grid, q = pre.grid(), pre.resolved()
    ids = processing_order(grid, 0)[:32]
    lo, hi = grid.decode(ids)
    groups = pa_groups(q, lo, hi)
    assert len(groups) > 1 and sorted(np.concatenate(groups).tolist()) == list(range(len(ids)))
    m = get_model("AC-8", weights="random", seed=1)
    be = Backend(m)
    bc = BaBConfig(node_budget=32)
    whole = BaBSolver(be, q, bc).solve(lo, hi, m)
    for g in groups:
        part = BaBSolver(be, q, bc).solve(lo[g], hi[g], m)
        assert np.array_equal(part.status, whole.status[g])
        assert np.array_equal(part.cex_x, whole.cex_x[g]) and np.array_equal(part.nodes, whole.nodes[g])
