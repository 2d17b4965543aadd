"""K10 kNN (fa_knn_kernel) and K13 activation deltas (fa_actdiff_kernel) vs plain references."""
import numpy as np
import pytest
import torch

from fairify_amd.models.mlp import random_mlp

pytestmark = pytest.mark.gpu


def _knn_ref(X: np.ndarray, k: int) -> np.ndarray:
    """Exact squared distances in float64, the row itself first, ties to the lower index."""
    X = X.astype(np.float64)
    d = ((X[:, None, :] - X[None, :, :]) ** 2).sum(-1)
    np.fill_diagonal(d, -1.0)
    return np.argsort(d, axis=1, kind="stable")[:, :k]


@pytest.mark.parametrize("n,d,k", [(1, 3, 1), (300, 13, 5), (1029, 20, 5), (700, 6, 10), (257, 64, 16)])
def test_knn_kernel_matches_reference_with_ties(cuda, n, d, k):
    from fairify_amd.ops import hip as H

    rng = np.random.default_rng(n + d)
    X = rng.integers(0, 4, size=(n, d)).astype(np.float32)      # many exact ties
    idx, dist = H.knn(torch.from_numpy(X).to(cuda), k)
    ref = _knn_ref(X, k)
    assert np.array_equal(idx.cpu().numpy(), ref)
    dref = ((X[:, None, :].astype(np.float64) - X[ref].astype(np.float64)) ** 2).sum(-1)
    assert np.array_equal(dist.cpu().numpy().astype(np.float64), dref)


def test_consistency_device_path(cuda):
    from fairify_amd.analysis.metrics import consistency

    rng = np.random.default_rng(3)
    X = rng.integers(0, 6, size=(900, 13)).astype(np.float32)
    y = rng.integers(0, 2, size=900).astype(np.float64)
    got = consistency(X, y, k=5, device=cuda, method="device")
    idx = _knn_ref(X, 5)
    ref = 1.0 - np.mean(np.abs(y - y[idx].mean(axis=1)))
    assert abs(got - ref) < 1e-6


@pytest.mark.parametrize("hidden", [[16, 8], [100, 100], [150, 100, 50, 25, 10, 5]])
def test_actdiff_kernel_matches_torch(cuda, hidden):
    from fairify_amd.repair.retrain import activation_deltas

    m = random_mlp(13, hidden, seed=len(hidden), bias_scale=0.3)
    rng = np.random.default_rng(0)
    x = rng.integers(0, 10, size=(501, 13)).astype(np.float64)
    xp = x.copy()
    xp[:, 8] = 1 - (x[:, 8] % 2)
    X = np.stack([x, xp], axis=1).reshape(-1, 13)
    X[7, 3] += 1          # one pair breaks the non-PA equality: dropped by both paths
    cpu = activation_deltas(m, X, 8, device="cpu")
    gpu = activation_deltas(m, X, 8, device=cuda)
    assert gpu.shape == cpu.shape == (m.n_neurons,)
    assert np.allclose(gpu, cpu, rtol=1e-4, atol=1e-5 * (1 + np.abs(cpu).max()))
