"""Buffer-lifetime rule of the multi-stream BaB path.

Round 1's profiled runs with 8 host threads / HIP streams crashed inside HIP copies.  The native
runtime then enqueued ``hipMemcpyAsync`` from pageable ``std::vector`` temporaries and, for
relaxed queries, rewrote a source vector in place right after enqueueing its copy (the x' boxes
were derived from the x boxes by editing ``hl``/``hh`` between two async copies).  A pageable
async H2D copy is staged by the HIP runtime after the call returns, so the second edit raced the
first copy.  The rule the runtime follows now (``csrc/bab_runtime.cpp``, ``ensure_host``):

* the host side of every ``hipMemcpyAsync`` is a runtime-owned pinned buffer (``hipHostMalloc``);
* such a buffer is only written, regrown or freed after the ``hipStreamSynchronize`` that
  retires the copy reading it.

The CPU test checks the first point on the source; the GPU test drives the former hazard (a
relaxed query, the x' pool path) from 8 threads with their own streams and runtimes and requires
the serial verdicts and counterexamples.
"""
import os
import re
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fairify_amd", "csrc")


def _host_operands(src: str):
    """(direction, host operand) of every hipMemcpyAsync call in ``src``."""
    out = []
    for m in re.finditer(r"hipMemcpyAsync\(([^;]*?)\)\s*,\s*\"", src, flags=re.S):
        args = [a.strip() for a in m.group(1).split(",")]
        kind = next(a for a in args if a.startswith("hipMemcpy"))
        host = args[1] if kind == "hipMemcpyHostToDevice" else args[0]
        out.append((kind, host))
    return out


RUNTIMES = ("bab_runtime.cpp", "relu_runtime.cpp", "beta_runtime.cpp")


def _pinned_names(src: str):
    """Runtime-owned pinned buffers: fa_mem::HostBuf members (csrc/devmem.h)."""
    names = set()
    for m in re.finditer(r"fa_mem::HostBuf\s+([^;]+);", src):
        for part in m.group(1).split(","):
            names.add(re.split(r"[{\s]", part.strip())[0])
    return names


def test_async_copies_use_pinned_runtime_buffers():
    for f in RUNTIMES:
        src = open(os.path.join(CSRC, f)).read()
        ops = _host_operands(src)
        assert len(ops) >= 3, (f, ops)
        pinned = _pinned_names(src)
        for kind, host in ops:
            if kind == "hipMemcpyDeviceToDevice":
                continue
            name = host.split("+")[0].strip()
            assert name.endswith(".p") and name[:-2] in pinned, \
                f"{f}: {kind} from/to {host!r} is not a runtime-owned pinned buffer"
            assert ".data()" not in host, host
        # no raw driver allocation / free in the runtimes: everything goes through the cache
        assert "hipHostFree" not in src and "hipFree(" not in src and "hipHostMalloc" not in src, f
    # no other source file enqueues async host copies (they go through torch or the runtimes)
    for f in os.listdir(CSRC):
        if f.endswith((".hip", ".cpp")) and f not in RUNTIMES:
            assert "hipMemcpyAsync" not in open(os.path.join(CSRC, f)).read(), f


def test_pinned_buffers_regrow_only_after_sync():
    """Every pinned-buffer regrowth (HostBuf::ensure, which releases the old block to the shared
    cache) is preceded, within the same function, by a stream synchronisation, or sits at the
    start of a solve (the previous solve ended with a sync), or is the D2H target that the
    synchronisation right after it retires."""
    for f in RUNTIMES:
        src = open(os.path.join(CSRC, f)).read()
        pinned = _pinned_names(src)
        body = src[src.index("py::tuple solve("):]
        first_sync = body.index("hipStreamSynchronize")
        for m in re.finditer(r"\b(\w+)\.ensure\(", body):
            if m.group(1) not in pinned:
                continue
            pos = m.start()
            fn_start = max(body.rfind("\n  void ", 0, pos), 0)
            before = body[fn_start:pos]
            at_solve_start = pos < first_sync and m.group(1) == "hstage_"
            # cand_host_ (candidate records the split kernel writes into pinned memory) regrows in
            # ensure_cand, called at a level start: the previous level ended with its stream sync
            # (and the constructor / solve start had no kernels in flight)
            # confirm_candidates runs right after the level-end sync (its caller), which retired the
            # previous level's copies from hidx_
            after_level_sync = "void confirm_candidates" in before and m.group(1) == "hidx_"
            assert at_solve_start or after_level_sync or "hipStreamSynchronize" in before \
                or m.group(1) in ("hout_", "hcand_") \
                or (m.group(1) == "cand_host_" and "void ensure_cand" in before), (f, m.group(1))


def test_runtime_pool_reuses_idle_runtimes():
    """engine/rtpool.py: an idle runtime of the same key is handed to the next caller whatever its
    thread; a larger capacity builds a new one and drops the outgrown idle ones."""
    import threading

    from fairify_amd.engine.rtpool import checkout, count

    class Owner:
        pass

    o, made = Owner(), []

    def make(cap):
        made.append(cap)
        return ("rt", cap, len(made))

    with checkout(o, "_p", "k", 10, make) as a:
        pass
    got, held = [], []

    def other_thread():
        cm = checkout(o, "_p", "k", 8, make)
        held.append(cm)                          # keep it checked out
        got.append(cm.__enter__())

    t = threading.Thread(target=other_thread)
    t.start()
    t.join()
    assert got[0] is a and made == [10]          # reused from another thread
    with checkout(o, "_p", "k", 10, make) as b:  # the first one is checked out: build another
        assert b is not a
    assert made == [10, 10]
    with checkout(o, "_p", "k", 40, make) as c:
        assert c[1] == 40
    assert count(o, "_p") == 1                   # the outgrown idle runtime was dropped


@pytest.mark.gpu
def test_relaxed_bab_eight_streams_match_serial(cuda):
    import torch

    from fairify_amd import presets
    from fairify_amd.engine.pipeline import VerifyConfig, verify_chunk
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend
    from fairify_amd.partition import processing_order

    pre = presets.get("relaxed/AC")
    grid, q = pre.grid(), pre.resolved()
    assert q.ra_idx and q.tau > 0
    order = processing_order(grid, 0)
    chunks = [order[i * 256:(i + 1) * 256] for i in range(8)]
    m = get_model("AC-3", weights="random", seed=0)
    be = Backend(m, cuda)
    cfg = VerifyConfig(sim_size=128, node_budget=256, smt_backend="none", residual_samples=256)
    serial = [verify_chunk(be, m, q, grid, ids, cfg) for ids in chunks]

    def run(ids):
        s = torch.cuda.Stream(cuda)
        with torch.cuda.stream(s):
            out = verify_chunk(be, m, q, grid, ids, cfg)
            torch.cuda.current_stream(cuda).synchronize()
        return out

    for _ in range(2):
        with ThreadPoolExecutor(8) as ex:
            conc = list(ex.map(run, chunks))
        for a, b in zip(serial, conc):
            assert np.array_equal(a.cols["verdict"], b.cols["verdict"])
            sat = a.cols["verdict"] == "sat"
            assert np.array_equal(a.cols["cex_x"][sat], b.cols["cex_x"][sat])
            assert np.array_equal(a.cols["cex_xp"][sat], b.cols["cex_xp"][sat])


@pytest.mark.gpu
def test_steady_state_issues_no_driver_frees(cuda):
    """After a first pass over a set of chunks (8 threads, pooled runtimes), running the same
    chunks again from other threads allocates nothing new from the driver and frees nothing:
    every runtime buffer comes out of the caching allocator (csrc/devmem.h)."""
    import torch

    from fairify_amd import presets
    from fairify_amd.engine.pipeline import VerifyConfig, verify_chunk
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops import ext
    from fairify_amd.ops.backend import Backend
    from fairify_amd.partition import processing_order

    pre = presets.get("src/AC-sex")
    grid, q = pre.grid(), pre.resolved()
    order = processing_order(grid, 0)
    m = get_model("AC-8", weights="random", seed=0)
    be = Backend(m, cuda)
    cfg = VerifyConfig(sim_size=128, node_budget=256, smt_backend="none", residual_samples=256, relu_budget=256)
    chunks = [order[i * 512:(i + 1) * 512] for i in range(8)]

    def run(ids):
        s = torch.cuda.Stream(cuda)
        with torch.cuda.stream(s):
            out = verify_chunk(be, m, q, grid, ids, cfg)
            torch.cuda.current_stream(cuda).synchronize()
        return out

    with ThreadPoolExecutor(8) as ex:
        first = list(ex.map(run, chunks))
    s0 = ext().mem_stats()
    with ThreadPoolExecutor(8) as ex:
        second = list(ex.map(run, chunks[::-1]))     # other threads get other chunks
    s1 = ext().mem_stats()
    for a, b in zip(first, second[::-1]):
        assert np.array_equal(a.cols["verdict"], b.cols["verdict"])
    assert s1["driver_frees"] == s0["driver_frees"] == 0, (s0, s1)
    assert s1["dev_hits"] >= s0["dev_hits"]
