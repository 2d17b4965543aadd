"""Multi-rank data-parallel verification over gloo (CPU): identical results to one rank."""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from fairify_amd.report.csv_report import read_csv


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch

    torch.set_num_threads(1)
    from fairify_amd import presets
    from fairify_amd.engine.pipeline import VerifyConfig
    from fairify_amd.engine.runner import run_preset
    from fairify_amd.parallel import dist as D

    info = D.init("cpu")
    cfg = VerifyConfig(sim_size=200, chunk=16, node_budget=512)
    run_preset(presets.get("src/GC-age"), models=["GC-1", "GC-4"], out_dir=out, cfg=cfg, info=info,
               max_partitions=70, accuracy=False, verbose=False)
    # collective helpers
    x = D.all_reduce_sum(info, np.array([rank + 1.0]))
    assert x[0] == sum(range(1, world + 1))
    g = D.all_gather_rows(info, np.full((rank + 1, 3), rank, dtype=np.int32))
    assert g.shape == (sum(range(1, world + 1)), 3)
    bits = D.pack_bits(np.eye(5, 11, dtype=bool))
    assert np.array_equal(D.unpack_bits(bits, 11), np.eye(5, 11, dtype=bool))
    D.destroy(info)


def _run(world, out):
    port = _free_port()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)


def test_two_ranks_match_one_rank(tmp_path):
    one, two = str(tmp_path / "one"), str(tmp_path / "two")
    _run(1, one)
    _run(2, two)
    for m in ["GC-1", "GC-4"]:
        a = read_csv(os.path.join(one, f"{m}.csv"))
        b = read_csv(os.path.join(two, f"{m}.csv"))
        assert len(a) == len(b) == 70
        for ra, rb in zip(a, b):
            for col in ["Partition_ID", "Verification", "SAT_count", "UNSAT_count", "UNK_count", "C1", "C2"]:
                assert ra[col] == rb[col], (m, col)
    s = json.load(open(os.path.join(two, "summary.json")))
    assert s["n_ranks"] == 2


def test_resume_skips_finished(tmp_path):
    from fairify_amd import presets
    from fairify_amd.engine.pipeline import VerifyConfig
    from fairify_amd.engine.runner import run_preset

    out = str(tmp_path / "r")
    cfg = VerifyConfig(sim_size=100, chunk=8, node_budget=256)
    pre = presets.get("src/GC-sex")
    run_preset(pre, models=["GC-3"], out_dir=out, cfg=cfg, max_partitions=20, accuracy=False, verbose=False)
    rows = run_preset(pre, models=["GC-3"], out_dir=out, cfg=cfg, max_partitions=40, resume=True,
                      accuracy=False, verbose=False)
    csv_rows = read_csv(os.path.join(out, "GC-3.csv"))
    assert len(csv_rows) == 40
    assert sorted(int(r["Partition_ID"]) for r in csv_rows) == list(range(1, 41))
    assert rows[0]["#P"] == 20          # this invocation verified only the new ones
