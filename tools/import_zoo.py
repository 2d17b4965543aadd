"""Convert the reference's Keras model zoo (models/*/*.h5) into the framework's .npz assets.

Uses the framework's own HDF5 reader (no h5py / TensorFlow); only weights are extracted.
Usage: python tools/import_zoo.py [/root/reference/models]
"""
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from fairify_amd.models.keras_io import load_keras_h5  # noqa: E402
from fairify_amd.models.zoo import ASSET_DIR, ZOO  # noqa: E402


def main(src: str) -> None:
    os.makedirs(ASSET_DIR, exist_ok=True)
    n = 0
    for path in sorted(glob.glob(os.path.join(src, "*", "*.h5"))):
        name = os.path.splitext(os.path.basename(path))[0]
        m = load_keras_h5(path, name=name)
        if name in ZOO:
            suite, n_in, hidden = ZOO[name]
            assert m.n_in == n_in and tuple(m.hidden) == hidden, (name, m.describe())
        m.save_npz(os.path.join(ASSET_DIR, f"{name}.npz"))
        n += 1
    print(f"imported {n} models into {ASSET_DIR}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/models")
