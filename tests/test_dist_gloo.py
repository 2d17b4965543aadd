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
    cfg = VerifyConfig(sim_size=200, chunk=16, node_budget=512, smt_backend="none")
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


_TIMES = {"SV-time", "S-time", "HV-Time", "H-Time", "Total-Time"}


def test_ranks_match_one_rank(tmp_path):
    """1, 2, 4 and 8 ranks (the CLI's dynamic unit queue for world > 1) write identical CSVs (every
    column but the measured times) through the compact rank-0 gather, and the per-rank partition
    counts of summary.json cover each model's partitions exactly once."""
    dirs = {w: str(tmp_path / f"w{w}") for w in (1, 2, 4, 8)}
    for w, d in dirs.items():
        _run(w, d)
    for m in ["GC-1", "GC-4"]:
        a = read_csv(os.path.join(dirs[1], f"{m}.csv"))
        assert len(a) == 70
        for w in (2, 4, 8):
            b = read_csv(os.path.join(dirs[w], f"{m}.csv"))
            assert len(b) == 70
            for ra, rb in zip(a, b):
                for col in ra:
                    if col not in _TIMES:
                        assert ra[col] == rb[col], (m, w, col)
    for w in (1, 2, 4, 8):
        s = json.load(open(os.path.join(dirs[w], "summary.json")))
        assert s["n_ranks"] == w
        rows = s["rows"] if "rows" in s else s["models"]
        for row in rows:
            assert len(row["rank_partitions"]) == w and sum(row["rank_partitions"]) == 70, (w, row["rank_partitions"])


def test_resume_skips_finished(tmp_path):
    from fairify_amd import presets
    from fairify_amd.engine.pipeline import VerifyConfig
    from fairify_amd.engine.runner import run_preset

    out = str(tmp_path / "r")
    cfg = VerifyConfig(sim_size=100, chunk=8, node_budget=256, smt_backend="none")
    pre = presets.get("src/GC-sex")
    run_preset(pre, models=["GC-3"], out_dir=out, cfg=cfg, max_partitions=20, accuracy=False, verbose=False)
    rows = run_preset(pre, models=["GC-3"], out_dir=out, cfg=cfg, max_partitions=40, resume=True,
                      accuracy=False, verbose=False)
    csv_rows = read_csv(os.path.join(out, "GC-3.csv"))
    assert len(csv_rows) == 40
    assert sorted(int(r["Partition_ID"]) for r in csv_rows) == list(range(1, 41))
    assert rows[0]["#P"] == 20          # this invocation verified only the new ones


def _worker_escalate(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch

    torch.set_num_threads(1)
    from fairify_amd import presets
    from fairify_amd.engine.pipeline import VerifyConfig
    from fairify_amd.engine.runner import run_preset
    from fairify_amd.parallel import dist as D

    info = D.init("cpu")
    cfg = VerifyConfig(sim_size=100, chunk=24, node_budget=16, heuristic=False, smt_backend="none")
    run_preset(presets.get("src/AC-sex"), models=["AC-7"], weights="random", out_dir=out, cfg=cfg, info=info,
               max_partitions=48, accuracy=False, verbose=False, escalate=8)
    D.destroy(info)


def test_residual_redistribution_matches_one_rank(tmp_path):
    """UNKNOWN partitions re-sharded over the ranks and retried with 8x budget: the result
    table is independent of the rank count."""
    one, two = str(tmp_path / "one"), str(tmp_path / "two")
    for w, out in ((1, one), (2, two)):
        port = _free_port()
        mp.spawn(_worker_escalate, args=(w, port, out), nprocs=w, join=True)
    a = read_csv(os.path.join(one, "AC-7.csv"))
    b = read_csv(os.path.join(two, "AC-7.csv"))
    assert len(a) == len(b) == 48
    for ra, rb in zip(a, b):
        for col in ["Partition_ID", "Verification", "C1", "C2"]:
            assert ra[col] == rb[col], col


def test_injected_crash_then_resume_matches_uninterrupted(tmp_path, monkeypatch):
    from fairify_amd import presets
    from fairify_amd.engine.pipeline import VerifyConfig
    from fairify_amd.engine.runner import run_preset
    from fairify_amd.utils.faults import InjectedFault

    pre = presets.get("src/GC-age")
    cfg = VerifyConfig(sim_size=100, chunk=8, node_budget=256, smt_backend="none")
    ref_dir, out = str(tmp_path / "ref"), str(tmp_path / "crash")
    run_preset(pre, models=["GC-4"], out_dir=ref_dir, cfg=cfg, max_partitions=40, accuracy=False, verbose=False)
    monkeypatch.setenv("FAIRIFY_FAULT_CRASH_AFTER", "2")
    with pytest.raises(InjectedFault):
        run_preset(pre, models=["GC-4"], out_dir=out, cfg=cfg, max_partitions=40, accuracy=False, verbose=False)
    assert len(read_csv(os.path.join(out, "GC-4.csv"))) == 16      # two checkpointed rounds of 8
    monkeypatch.delenv("FAIRIFY_FAULT_CRASH_AFTER")
    run_preset(pre, models=["GC-4"], out_dir=out, cfg=cfg, max_partitions=40, resume=True, accuracy=False,
               verbose=False)
    a = read_csv(os.path.join(ref_dir, "GC-4.csv"))
    b = read_csv(os.path.join(out, "GC-4.csv"))
    assert len(a) == len(b) == 40
    for ra, rb in zip(a, b):
        for col in ["Partition_ID", "Verification", "SAT_count", "UNSAT_count", "UNK_count", "C1", "C2"]:
            assert ra[col] == rb[col], col


def test_forced_unknown_injection(monkeypatch):
    from fairify_amd import presets
    from fairify_amd.engine.pipeline import VerifyConfig, verify_chunk
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend
    from fairify_amd.partition import processing_order
    from fairify_amd.utils.faults import forced_unknown

    pre = presets.get("src/GC-age")
    grid, q = pre.grid(), pre.resolved()
    ids = processing_order(grid, 0)[:32]
    m = get_model("GC-4")
    cfg = VerifyConfig(sim_size=100, node_budget=256, heuristic=False, smt_backend="none")
    base = [r["verdict"] for r in verify_chunk(Backend(m), m, q, grid, ids, cfg)]
    monkeypatch.setenv("FAIRIFY_FAULT_FORCE_UNKNOWN", "0.5")
    mask = forced_unknown(ids)
    assert 0 < mask.sum() < len(ids)
    recs = verify_chunk(Backend(m), m, q, grid, ids, cfg)
    for r, b, f in zip(recs, base, mask):
        if f and r["stage"] != "sim" and b != "unknown":
            assert r["verdict"] == "unknown"
        elif not f:
            assert r["verdict"] == b


def test_wire_roundtrip_and_size():
    """Compact per-partition wire records: exact round trip, <= 32 B per Adult partition."""
    from fairify_amd import presets
    from fairify_amd.engine.pipeline import ChunkRecords
    from fairify_amd.parallel import wire

    q = presets.get("src/AC-sex").resolved()
    rng = np.random.default_rng(0)
    n, N, S = 4096, 201, 1000
    verdict = rng.choice(np.array(["sat", "unsat", "unknown"]), size=n, p=[0.25, 0.7, 0.05])
    sat = verdict == "sat"
    cx = np.where(sat[:, None], rng.integers(0, 90, size=(n, q.n)), 0)
    cxp = cx.copy()
    cxp[sat, q.pa_idx[0]] = 1 - cx[sat, q.pa_idx[0]]
    core = dict(grid_id=np.arange(n), verdict=verdict, stage=rng.choice(np.array(wire.STAGES[1:], dtype=object), n),
                h_attempt=rng.integers(0, 2, n), h_success=rng.integers(0, 2, n),
                b_cnt=rng.integers(0, N, n), s_cnt=rng.integers(0, N, n), st_cnt=rng.integers(0, N, n),
                h_cnt=rng.integers(0, N, n), t_cnt=rng.integers(0, N, n), agree=rng.integers(0, S + 1, n),
                tp=rng.integers(0, S // 2, n), fp=rng.integers(0, S // 4, n), nodes=rng.integers(0, 1 << 20, n), c_check=rng.integers(0, 2, n), v_accurate=rng.integers(0, 2, n),
                cex_x=cx, cex_xp=cxp)
    recs = ChunkRecords(core, 0.8, segments=[(1000, 1.0, 0.5, 0.1, 0.01), (n - 1000, 2.0, 1.5, 0.0, 0.02)],
                        n_neurons=N, sim_size=S)
    buf = wire.encode(recs, q)
    assert len(buf) / n <= 32.0, len(buf) / n
    back = wire.decode(buf, np.arange(n), 0.8, N, S, q)
    for k, v in recs.cols.items():
        if v.dtype.kind in "OU":
            assert list(back.cols[k]) == list(v), k
        else:
            assert np.array_equal(back.cols[k], v), k


def _claim_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import threading

    from fairify_amd.engine.runner import _claim_fn
    from fairify_amd.parallel import dist as D

    info = D.init("cpu")
    claim = _claim_fn(info)
    got = []
    lock = threading.Lock()

    def th():
        while True:
            u = claim("fairify/test/units")
            if u >= 200:
                return
            with lock:
                got.append(u)

    ts = [threading.Thread(target=th) for _ in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    all_units = D.all_gather_rows(info, np.asarray(sorted(got), np.int64).reshape(-1, 1)).reshape(-1)
    if rank == 0:
        q.put(sorted(all_units.tolist()))
    D.destroy(info)


@pytest.mark.parametrize("world", [4, 8])
def test_unit_queue_claims_every_unit_once(world):
    """The runner's dynamic unit queue (rendezvous-store atomic counter): 4 / 8 ranks x 3 threads
    claim 200 units, each exactly once."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    mp.spawn(_claim_worker, args=(world, port, q), nprocs=world, join=True)
    assert q.get() == list(range(200))


def _worker_twice(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch

    torch.set_num_threads(1)
    from fairify_amd import presets
    from fairify_amd.engine.pipeline import VerifyConfig
    from fairify_amd.engine.runner import run_preset
    from fairify_amd.parallel import dist as D

    info = D.init("cpu")
    cfg = VerifyConfig(sim_size=100, chunk=8, node_budget=256, smt_backend="none")
    for k in range(2):
        run_preset(presets.get("src/GC-age"), models=["GC-4"], out_dir=os.path.join(out, str(k)), cfg=cfg, info=info,
                   max_partitions=40, accuracy=False, verbose=False, balance="queue")
    D.destroy(info)


def test_unit_queue_second_run_same_process_group(tmp_path):
    """A second run_preset of the same preset / model / seed in one process group gets fresh unit
    counters (per-invocation nonce) and verifies every partition again (the stale key used to drop
    the whole run silently)."""
    port = _free_port()
    mp.spawn(_worker_twice, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    a = read_csv(os.path.join(str(tmp_path), "0", "GC-4.csv"))
    b = read_csv(os.path.join(str(tmp_path), "1", "GC-4.csv"))
    assert len(a) == len(b) == 40
    for ra, rb in zip(a, b):
        for col in ra:
            if col not in _TIMES:
                assert ra[col] == rb[col], col


def test_strided_and_queue_balance_agree(tmp_path):
    """--balance strided and the default queue write the same verdict columns at 2 ranks."""
    outs = {}
    for bal in ("queue", "strided"):
        d = str(tmp_path / bal)
        port = _free_port()
        mp.spawn(_worker_bal, args=(2, port, d, bal), nprocs=2, join=True)
        outs[bal] = read_csv(os.path.join(d, "GC-4.csv"))
    a, b = outs["queue"], outs["strided"]
    assert len(a) == len(b) == 40
    for ra, rb in zip(a, b):
        for col in ra:
            if col not in _TIMES:
                assert ra[col] == rb[col], col
    s = json.load(open(os.path.join(str(tmp_path / "queue"), "summary.json")))
    row = s["rows"][0] if "rows" in s else s["models"][0]
    assert row["balance"] == "queue" and sum(row["rank_partitions"]) == 40


def _worker_bal(rank, world, port, out, bal):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch

    torch.set_num_threads(1)
    from fairify_amd import presets
    from fairify_amd.engine.pipeline import VerifyConfig
    from fairify_amd.engine.runner import run_preset
    from fairify_amd.parallel import dist as D

    info = D.init("cpu")
    cfg = VerifyConfig(sim_size=100, chunk=8, node_budget=256, smt_backend="none")
    run_preset(presets.get("src/GC-age"), models=["GC-4"], out_dir=out, cfg=cfg, info=info, max_partitions=40,
               accuracy=False, verbose=False, balance=bal)
    D.destroy(info)
