"""Distributed paths on a real GPU box (one MI355X): the RCCL communicator (a one-rank process
group, since RCCL refuses two ranks on one device) and the self-launching bench with two ranks
sharing the GPU over gloo."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench_json(args, env):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       env=env, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


SMALL = ["--models", "AC-8,AC-3", "--limit", "2048", "--steps", "1", "--warmup", "1"]


def test_rccl_one_rank_bench(cuda):
    env = dict(os.environ, FAIRIFY_DIST_INIT="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    env.pop("FAIRIFY_DIST_BACKEND", None)
    d = _bench_json(["--gpus", "1", *SMALL], env)
    assert d["dist"]["backend"] == "nccl" and d["n_gpus"] == 1
    base = _bench_json(["--gpus", "1", *SMALL], {k: v for k, v in os.environ.items() if k != "WORLD_SIZE"})
    for k in ("sat", "unsat", "unknown"):
        assert d[k] == base[k], k


def test_self_launch_two_ranks_share_gpu(cuda):
    env = dict(os.environ, FAIRIFY_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    one = _bench_json(["--gpus", "1", *SMALL], env)
    two = _bench_json(["--gpus", "2", "--concurrency", "2", *SMALL], env)
    assert two["n_gpus"] == 2 and two["dist"]["backend"] == "gloo" and len(two["dist"]["rank_ms_per_step"]) == 2
    for k in ("sat", "unsat", "unknown", "unsat_sound", "unsat_heuristic"):
        assert one[k] == two[k], k


def test_rccl_collectives_one_rank(cuda):
    code = r'''
import os, numpy as np
from fairify_amd.parallel import dist as D
info = D.init("cuda")
assert D.backend_name(info) == "nccl", D.backend_name(info)
buf = np.arange(1000, dtype=np.uint8)
h = D.gather_bytes(info, buf, async_op=True)
out = h.wait()
assert len(out) == 1 and np.array_equal(out[0], buf)
assert np.array_equal(D.all_gather_int8(info, np.array([1, 0, 2], np.int8)), [1, 0, 2])
assert D.all_reduce_sum(info, np.array([2.0]))[0] == 2.0
assert D.all_gather_floats(info, 3.5) == [3.5]
D.barrier(info)
D.destroy(info)
print("ok")
'''
    env = dict(os.environ, FAIRIFY_DIST_INIT="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), PYTHONPATH=ROOT)
    env.pop("FAIRIFY_DIST_BACKEND", None)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120, cwd=ROOT)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-3000:]
