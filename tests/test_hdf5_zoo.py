"""Own HDF5 reader vs shipped weights; zoo architectures."""
import glob
import os
import subprocess

import numpy as np
import pytest

from fairify_amd.models.zoo import SUITE_MODELS, ZOO, get_model, has_weights

REF = "/root/reference/models"


def test_zoo_shapes():
    assert len(ZOO) >= 53
    for name, (suite, n_in, hidden) in ZOO.items():
        m = get_model(name, weights="random")
        assert m.n_in == n_in and tuple(m.hidden) == hidden
        if has_weights(name):
            z = get_model(name)
            assert z.n_in == n_in and tuple(z.hidden) == hidden


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference models not mounted")
def test_reader_matches_assets():
    from fairify_amd.models.keras_io import load_keras_h5

    for path in sorted(glob.glob(os.path.join(REF, "*", "*.h5"))):
        name = os.path.basename(path)[:-3]
        a = load_keras_h5(path)
        b = get_model(name)
        for wa, wb in zip(a.weights + a.biases, b.weights + b.biases):
            assert np.array_equal(wa, wb)


H5PY = "/opt/conda/bin/python3.9"


@pytest.mark.skipif(not (os.path.isdir(REF) and os.path.exists(H5PY)), reason="no h5py oracle")
def test_reader_matches_h5py_oracle():
    from fairify_amd.models.keras_io import load_keras_h5

    script = (
        "import h5py,sys,numpy as np\n"
        "f=h5py.File(sys.argv[1],'r');mw=f['model_weights'];s=0.0\n"
        "for ln in mw.attrs['layer_names']:\n"
        "  ln=ln.decode() if isinstance(ln,bytes) else ln;g=mw[ln]\n"
        "  for w in g.attrs['weight_names']:\n"
        "    w=w.decode() if isinstance(w,bytes) else w;s+=float(np.abs(g[w][()]).astype(np.float64).sum())\n"
        "print(repr(s))\n")
    for path in sorted(glob.glob(os.path.join(REF, "*", "*.h5")))[::7]:
        out = subprocess.run([H5PY, "-c", script, path], capture_output=True, text=True, env={})
        if out.returncode != 0:
            pytest.skip("h5py oracle unavailable: " + out.stderr[-200:])
        m = load_keras_h5(path)
        s = sum(float(np.abs(x).astype(np.float64).sum()) for x in m.weights + m.biases)
        assert abs(s - float(out.stdout.strip())) <= 1e-9 * max(1.0, s)


def test_npz_roundtrip(tmp_path):
    m = get_model("BM-4", weights="random", seed=3)
    p = tmp_path / "m.npz"
    m.save_npz(str(p))
    from fairify_amd.models.mlp import MLP

    m2 = MLP.load_npz(str(p))
    assert all(np.array_equal(a, b) for a, b in zip(m.weights, m2.weights))


def test_prune_equals_masked_forward():
    m = get_model("AC-4", weights="random", seed=1)
    rng = np.random.default_rng(0)
    dead = [rng.random(w) < 0.3 for w in m.widths[:-1]] + [np.zeros(1, bool)]
    x = rng.integers(0, 20, size=(64, 13))
    assert np.allclose(m.prune(dead).logits(x), m.masked(dead).logits(x), atol=1e-9)
