"""HIP pruning-stage kernels (csrc/prune.hip) against the PyTorch mask algebra they replace
(engine/prune.py) -- exact equality -- and the Pruned-acc agreement kernel against rigorous
point bounds."""
import numpy as np
import pytest
import torch

from fairify_amd.engine import prune as P_
from fairify_amd.models.mlp import random_mlp
from fairify_amd.ops.backend import Backend

pytestmark = pytest.mark.gpu


def _inputs(m, P, seed, dev):
    g = torch.Generator().manual_seed(seed)
    N, Nh = m.n_neurons, int(sum(m.hidden))
    counts = torch.randint(0, 3, (P, N), generator=g, dtype=torch.int32)
    counts[torch.rand(P, N, generator=g) < 0.3] = 0
    counts[: P // 8] = 0                                  # whole layers of candidates
    ub = torch.randn(P, N, generator=g) * 2.0
    lb = ub - torch.rand(P, N, generator=g) * 3.0
    ub[P // 8: P // 4] = -torch.rand(P // 4 - P // 8, N, generator=g)   # whole layers bound-dead
    sd = (torch.rand(P, Nh, generator=g) < 0.4).to(torch.uint8)
    return counts.to(dev), lb.to(dev), ub.to(dev), sd.to(dev)


@pytest.mark.parametrize("hidden", [[16, 8], [100, 100], [5, 5, 5, 5], [64, 32, 16, 8, 4]])
def test_prune_masks_and_heuristic_match_torch(cuda, hidden):
    from fairify_amd.ops import hip as H

    m = random_mlp(13, hidden, seed=3)
    be = Backend(m, cuda)
    widths = m.widths
    Nh = int(sum(m.hidden))
    P = 512
    counts, lb, ub, sd = _inputs(m, P, 7, cuda)
    code, cnt = H.prune_masks(be, counts, ub, sd)
    # PyTorch path (engine/pipeline.py, FAIRIFY_FUSED_PRUNE=0)
    cand, _ = P_.candidates_from_counts(counts, 1000)
    b_dead, b_rem = P_.bound_dead(cand, ub[:, :Nh], widths)
    b_dead = P_.ensure_one_alive(b_dead, widths)
    s_hid = b_rem[:, :Nh] & sd.bool()
    s_dead = torch.zeros_like(b_dead)
    s_dead[:, :Nh] = s_hid
    s_cand = b_rem.clone()
    s_cand[:, :Nh] = b_rem[:, :Nh] & ~s_hid
    st_dead = P_.ensure_one_alive(P_.merge(b_dead, s_dead), widths)
    bit = lambda b: (code & b) != 0
    assert torch.equal(bit(H.PM_CAND), cand)
    assert torch.equal(bit(H.PM_B), b_dead)
    assert torch.equal(bit(H.PM_S), s_dead)
    assert torch.equal(bit(H.PM_ST), st_dead)
    assert torch.equal(bit(H.PM_SCAND), s_cand)
    assert torch.equal(cnt.long(), torch.stack([b_dead.sum(1), s_dead.sum(1), st_dead.sum(1)], 1))
    # heuristic pruning on a subset of rows
    rows = torch.arange(0, P, 3, device=cuda)
    for perc in (5.0, 20.0):
        hn, hm, hc = H.heuristic(be, rows, lb, ub, code, perc)
        tn, tm_ = P_.heuristic_prune_batch(lb[rows], ub[rows], cand[rows], s_cand[rows], st_dead[rows], widths, perc)
        assert torch.equal(hn.bool(), tn), f"new masks differ (perc {perc})"
        assert torch.equal(hm.bool(), tm_), f"merged masks differ (perc {perc})"
        assert torch.equal(hc.long(), torch.stack([tn.sum(1), tm_.sum(1)], 1))
        assert int(tn.sum()) > 0   # the test exercises actual pruning


@pytest.mark.parametrize("hidden", [[16, 8], [100, 100], [64, 32, 16, 8, 4]])
def test_agree_kernel_within_rounding(cuda, hidden):
    """Agreement count of the full vs the masked network on the simulation points, bracketed by
    the points whose signs are certain under rigorous fp32 bounds."""
    from fairify_amd.ops import hip as H
    from fairify_amd.ops.reference import sample_points

    m = random_mlp(13, hidden, seed=11, bias_scale=0.3)
    be = Backend(m, cuda)
    Nh = int(sum(m.hidden))
    P, S = 40, 1000
    g = torch.Generator().manual_seed(5)
    lo = torch.randint(0, 20, (P, 13), generator=g).float()
    hi = lo + torch.randint(0, 10, (P, 13), generator=g).float()
    pids = torch.arange(100, 100 + P)
    rows = torch.arange(0, P, 2)
    dm = (torch.rand(rows.numel(), Nh, generator=g) < 0.3).to(torch.uint8)
    ag = H.agree(be, rows.to(cuda), lo.to(cuda), hi.to(cuda), pids.to(cuda), dm.to(cuda), S, 9)
    assert ag is not None
    X = sample_points(lo[rows], hi[rows], pids[rows], S, 9).to(cuda)
    R = X.shape[0] * S
    xf = X.reshape(R, 13)
    l0, u0 = be.point_bounds(xf)
    l1, u1 = be.point_bounds(xf, dm.to(cuda).repeat_interleave(S, 0))
    s0 = torch.where(l0 > 0, 1, torch.where(u0 < 0, -1, 0)).view(-1, S)
    s1 = torch.where(l1 > 0, 1, torch.where(u1 < 0, -1, 0)).view(-1, S)
    sure = (s0 != 0) & (s1 != 0)
    lo_cnt = (sure & (s0 == s1)).sum(1)
    hi_cnt = lo_cnt + (~sure).sum(1)
    a = ag[:, 0].long()
    assert bool(((a >= lo_cnt) & (a <= hi_cnt)).all())
    # true / false positives of the pruned labels, bracketed the same way
    tp_lo = (sure & (s0 > 0) & (s1 > 0)).sum(1)
    fp_lo = (sure & (s0 < 0) & (s1 > 0)).sum(1)
    unsure = (~sure).sum(1)
    tp, fp = ag[:, 1].long(), ag[:, 2].long()
    assert bool(((tp >= tp_lo) & (tp <= tp_lo + unsure) & (fp >= fp_lo) & (fp <= fp_lo + unsure)).all())
    assert int((~sure).sum()) < 0.01 * R
