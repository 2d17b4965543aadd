"""Partition grid: counts of every preset, reference order, decode/encode, order."""
import numpy as np
import pytest

from fairify_amd import presets
from fairify_amd.partition import Grid, permute, processing_order, reference_partition_list, shard
from fairify_amd.spec import ADULT, GERMAN, Domain, Feature

EXPECTED = {
    "src/AC-sex": 16000, "src/AC-race": 16000, "src/GC-age": 201, "src/GC-sex": 201, "src/BM-age": 510,
    "src/CP": 8, "src/DF": 8, "stress/AC": 3290112, "stress/GC": 18009, "stress/BM": 1002000,
    "relaxed/AC": 3290112, "relaxed/GC": 18009, "relaxed/BM": 1002000, "targeted/AC": 205632,
    "targeted/GC": 18009, "targeted/BM": 501000, "targeted2/AC": 1096704, "targeted2/GC": 18009,
    "targeted2/BM": 1002000, "experiment/AC-3": 32, "experiment/GC-1": 201, "experiment/BM": 1002000,
}


@pytest.mark.parametrize("name,count", sorted(EXPECTED.items()))
def test_preset_partition_counts(name, count):
    assert len(presets.get(name).grid()) == count


def test_decode_matches_reference_product_order():
    g = Grid.reference(GERMAN, 100)
    ref = reference_partition_list(GERMAN.range_dict(), 100)
    assert len(ref) == len(g)
    lo, hi = g.decode(np.arange(len(g)))
    for pid in [0, 1, 57, 200]:
        for i, f in enumerate(GERMAN.features):
            assert [lo[pid, i], hi[pid, i]] == ref[pid][f.name]


def test_decode_encode_roundtrip_and_cover():
    g = Grid.reference(ADULT, 10)
    ids = np.random.default_rng(0).choice(len(g), 500, replace=False)
    lo, hi = g.decode(ids)
    rng = np.random.default_rng(1)
    pts = rng.integers(lo, hi + 1)
    assert np.array_equal(g.encode(pts), ids)
    outside = pts.copy()
    outside[:, 0] = 1000
    assert np.all(g.encode(outside) == -1)


def test_boxes_tile_the_domain():
    dom = Domain("t", (Feature("a", 0, 9), Feature("b", 1, 7), Feature("c", 0, 2)))
    g = Grid.reference(dom, 3)
    lo, hi = g.decode(np.arange(len(g)))
    vol = np.prod(hi - lo + 1, axis=1).sum()
    assert vol == 10 * 7 * 3


def test_permutation_is_bijective_and_seeded():
    for n in [1, 2, 7, 1000, 16000, 3290112]:
        idx = np.arange(min(n, 20000))
        p = permute(idx, n, seed=3)
        assert p.min() >= 0 and p.max() < n
        assert len(np.unique(p)) == len(p)
    full = permute(np.arange(16000), 16000, 5)
    assert np.array_equal(np.sort(full), np.arange(16000))
    assert not np.array_equal(full, permute(np.arange(16000), 16000, 6))


def test_shards_partition_the_order():
    g = Grid.reference(GERMAN, 10)
    order = processing_order(g, seed=1)
    parts = [shard(order, r, 4) for r in range(4)]
    assert sorted(np.concatenate(parts).tolist()) == sorted(order.tolist())


def test_capped_partitioner_reference_semantics():
    g = presets.get("src/DF").grid()
    assert len(g) == 8
    assert [a.index for a in g.attrs] == [1]          # only AGE is split (LIMIT_BAL too large)
    lo, hi = g.decode(np.arange(8))
    assert lo[:, 1].min() == 21 and hi[:, 1].max() == 79


def test_columnar_csv_matches_record_writer(tmp_path):
    """The runner's columnar CSV path writes exactly the bytes of the per-record writer."""
    import numpy as np

    from fairify_amd.engine.runner import _SCALARS, columns, csv_layout, unpack
    from fairify_amd.report.csv_report import PartitionCSV

    rng = np.random.default_rng(3)
    n0, R = 13, 400
    rows = np.zeros((R, 4 + len(_SCALARS) + 1 + 2 * n0))
    rows[:, 0] = np.arange(R)
    rows[:, 1] = rng.integers(0, 10 ** 6, R)
    rows[:, 2] = rng.integers(0, 3, R)
    rows[:, 4:4 + len(_SCALARS)] = rng.random((R, len(_SCALARS)))
    rows[:, 4] = rng.integers(0, 2, R)
    rows[:, 5] = rng.integers(0, 2, R)
    sat = rows[:, 2] == 1
    rows[sat, 4 + len(_SCALARS)] = 1
    rows[sat, 5 + len(_SCALARS):] = rng.integers(0, 100, (int(sat.sum()), 2 * n0))
    rows[sat, 5 + len(_SCALARS) + 3] = 20000.0        # exponent-notation array on some rows
    rows[::7, 5 + len(_SCALARS) + 1] = -3.0
    rows[::5, 4 + 7] = 1e-7                          # repr in exponent notation
    rows[::6, 4 + 8] = 123456.0                      # integral float -> "123456.0"
    rows[::13, 4 + 2] = -0.0
    for acc in (None, 0.8123456):
        a, b, c, d = (tmp_path / f"{k}{acc}.csv" for k in "abcd")
        wa, wb, wc, wd = PartitionCSV(str(a)), PartitionCSV(str(b)), PartitionCSV(str(c)), PartitionCSV(str(d))
        for half in (rows[:150], rows[150:]):
            wa.write(unpack(half, n0, acc))
            wb.write_columns(columns(half, n0), acc)
            wc.write_packed(half, csv_layout(n0), n0, acc)                 # native formatter
            wd.write_packed(half, csv_layout(n0), n0, acc, native=False)
        assert a.read_bytes() == b.read_bytes() == c.read_bytes() == d.read_bytes()
        assert wa.counts == wb.counts == wc.counts == wd.counts
