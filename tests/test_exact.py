"""Exact sign of the logit (counterexample confirmation): fp64 + rigorous bound vs Fraction."""
import numpy as np

from fairify_amd.engine import exact
from fairify_amd.models.mlp import MLP, random_mlp


def _frac_sign(net, x):
    v = exact.exact_logit_fraction(net, x)
    return (v > 0) - (v < 0)


def test_signs_match_fraction_including_exact_zeros():
    rng = np.random.default_rng(0)
    zeros = 0
    for t in range(40):
        net = random_mlp(6, [5] * (1 + t % 4), seed=t, bias_scale=0.0 if t % 2 else 0.3)
        X = rng.integers(-3, 4, size=(50, 6))
        s = exact.exact_signs(net, X)
        ref = np.array([_frac_sign(net, x) for x in X])
        assert np.array_equal(s, ref), t
        zeros += int((ref == 0).sum())
    assert zeros > 0          # zero-bias nets with dead layers give exact-zero logits


def test_dead_layer_decided_without_fraction(monkeypatch):
    """A certainly-dead hidden layer makes the logit exactly 0: decided in fp64 (no Fraction)."""
    W1 = -np.ones((3, 4), np.float32)
    net = MLP([W1, np.ones((4, 1), np.float32)], [np.zeros(4, np.float32), np.zeros(1, np.float32)], name="d")
    monkeypatch.setattr(exact, "exact_logit_fraction", lambda *a: (_ for _ in ()).throw(AssertionError("slow path")))
    assert exact.exact_signs(net, np.array([[1, 2, 3], [0, 0, 1]])).tolist() == [0, 0]
    assert not exact.is_violation(net, np.array([[1, 2, 3]]), np.array([[1, 2, 4]]))[0]
