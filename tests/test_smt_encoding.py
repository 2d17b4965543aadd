"""SMT-LIB2 encoding of the partition query vs exact semantics (no solver needed).

The reference's Z3 query (src/AC/Verify-AC.py:127-158) is re-created as SMT-LIB2 text; here
an exact S-expression evaluator checks, on every lattice pair of tiny boxes, that the encoded
formula is satisfied exactly by the fairness violations (brute force on the exact network).
Z3 itself is absent in this image, so solver parity is "unpinned"; the encoding is pinned.
"""
import itertools

import numpy as np
import pytest
import torch

from fairify_amd.engine import exact
from fairify_amd.models.mlp import random_mlp
from fairify_amd.ops import reference as ref
from fairify_amd.smt import Evaluator, available, encode_partition, model_to_pair, parse_model, pruned_network
from fairify_amd.smt.host import HostSMT
from fairify_amd.spec import Domain, Feature, Query

DOM = Domain("toy", tuple(Feature(f"f{i}", 0, w) for i, w in enumerate([2, 3, 1, 2])))


def _assign(x, xp):
    d = {f"x{i}": int(v) for i, v in enumerate(x)}
    d.update({f"x_{i}": int(v) for i, v in enumerate(xp)})
    return d


@pytest.mark.parametrize("pa,ra,tau", [(("f2",), (), 0), (("f2",), ("f1",), 1), (("f2", "f0"), (), 0)])
def test_encoding_accepts_exactly_the_violations(pa, ra, tau):
    q = Query(pa=pa, ra=ra, tau=tau).resolve(DOM)
    lo, hi = np.zeros(4, int), np.array([2, 3, 1, 2])
    m = random_mlp(4, [5, 3], seed=17, bias_scale=1.0)
    ev = Evaluator(encode_partition(m, q, lo, hi).text)
    pts = np.array(list(itertools.product(*[range(a, b + 1) for a, b in zip(lo, hi)])))
    s = dict(zip(map(tuple, pts), exact.exact_signs(m, pts)))
    n_true = 0
    # x' ranges over the box widened by tau on relaxed attributes (they may leave the box)
    wide = [range(a - (tau if i in q.ra_idx else 0), b + 1 + (tau if i in q.ra_idx else 0))
            for i, (a, b) in enumerate(zip(lo, hi))]
    for x in pts:
        for xp in itertools.product(*wide):
            xp = np.array(xp)
            sat = ev.satisfied(_assign(x, xp))
            ok = exact.check_pair_constraints(x[None], xp[None], lo[None], hi[None], q.pa_idx, q.ra_idx, tau)[0]
            if ok:
                sp = exact.exact_signs(m, xp[None])[0]
                truth = bool(s[tuple(x)] * sp < 0)
            else:
                truth = False
            assert sat == truth, (x, xp)
            n_true += truth
    assert n_true > 0   # the toy net is unfair somewhere: the check is not vacuous


def test_encoded_logit_is_exact():
    q = Query(pa=("f2",)).resolve(DOM)
    m = random_mlp(4, [6, 4], seed=3, bias_scale=0.5)
    ev = Evaluator(encode_partition(m, q, [0, 0, 0, 0], [2, 3, 1, 2]).text)
    for x in [(0, 0, 0, 0), (2, 3, 1, 2), (1, 2, 0, 1)]:
        y = ev.eval_name("y", _assign(x, x))
        assert abs(float(y) - m.logits(np.array([x], dtype=np.float64))[0]) < 1e-9


def test_pruned_subnetwork_encoding_equivalent_on_box():
    """Sound pruning (neurons dead on the whole box) does not change the encoded function there."""
    q = Query(pa=("f2",)).resolve(DOM)
    m = random_mlp(4, [12, 6], seed=5, bias_scale=0.5)
    m.biases[0] = m.biases[0] - np.float32(2.0)    # push some first-layer neurons dead on the box
    lo, hi = np.array([0, 0, 0, 0]), np.array([2, 3, 1, 2])
    r = ref.bounds([torch.from_numpy(w).double() for w in m.weights], [torch.from_numpy(b).double() for b in m.biases],
                   torch.tensor(lo[None], dtype=torch.float64), torch.tensor(hi[None], dtype=torch.float64),
                   mode="ibp", keep_layers=True)
    dead = torch.cat([u <= 0 for u in r.layer_ub[:-1]], dim=1)[0].numpy()
    assert dead.any()
    pm = pruned_network(m, dead)
    assert pm.n_neurons < m.n_neurons
    ev_full = Evaluator(encode_partition(m, q, lo, hi).text)
    ev_pr = Evaluator(encode_partition(pm, q, lo, hi).text)
    for x in itertools.product(*[range(a, b + 1) for a, b in zip(lo, hi)]):
        a = _assign(x, x)
        assert ev_full.eval_name("y", a) == ev_pr.eval_name("y", a)


def test_parse_model_and_pair():
    out = """sat
(
  (define-fun x1 () Int
    3)
  (define-fun x_0 () Int
    (- 2))
  (define-fun x0 () Int
    7)
  (define-fun y () Real 0.5)
)"""
    body = out.split("\n", 1)[1]
    m = parse_model(body)
    assert m == {"x1": 3, "x_0": -2, "x0": 7}
    x, xp = model_to_pair(m, 2)
    assert x == [7, 3] and xp == [-2, 0]


def test_solver_backends_absent_here():
    """No Z3 in this image: ``auto`` resolves to the HiGHS MILP back-end (SciPy), which the
    pipeline drives directly (HostSMT, the SMT-LIB path, stays inactive for it)."""
    from fairify_amd.smt import milp
    from fairify_amd.smt.solver import resolve

    have = available()
    assert all(b in ("z3py", "z3bin", "milp") for b in have)
    if not any(b in ("z3py", "z3bin") for b in have):
        assert resolve("auto") == ("milp" if milp.available() else "none")
        with pytest.raises(RuntimeError):
            HostSMT("z3bin")
