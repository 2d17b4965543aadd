#!/usr/bin/env python
"""Count PyTorch ops (each one is at least one device dispatch on the GPU) per pipeline stage
for one bench work item (one model x one chunk), to find the torch glue worth fusing.

    python tools/count_ops.py [--model AC-7] [--chunk 4096] [--device cuda]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
from torch.utils._python_dispatch import TorchDispatchMode

from fairify_amd.utils import timer as T

_tls = threading.local()
_orig_call = T.StageTimer.__call__


class _Stage:
    def __init__(self, inner, name):
        self.inner, self.name = inner, name

    def __enter__(self):
        st = getattr(_tls, "stack", [])
        _tls.stack = st + [self.name]
        return self.inner.__enter__()

    def __exit__(self, *a):
        _tls.stack = _tls.stack[:-1]
        return self.inner.__exit__(*a)


def _call(self, name):
    return _Stage(_orig_call(self, name), name)


T.StageTimer.__call__ = _call


class Count(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.c = collections.Counter()
        self.ops = collections.defaultdict(collections.Counter)

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        st = "/".join(getattr(_tls, "stack", [])) or "(outside stages)"
        self.c[st] += 1
        self.ops[st][str(func.overloadpacket.__name__)] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="AC-7")
    ap.add_argument("--chunk", type=int, default=4096)
    ap.add_argument("--device", default="cuda" if torch.cuda.device_count() else "cpu")
    a = ap.parse_args()
    from fairify_amd import presets
    from fairify_amd.engine.pipeline import VerifyConfig, verify_chunk
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend
    from fairify_amd.partition import processing_order

    pre = presets.get("src/AC-sex")
    grid = pre.grid()
    q = pre.resolved()
    order = processing_order(grid, seed=0)
    m = get_model(a.model, weights="random", seed=0)
    be = Backend(m, device=torch.device(a.device))
    cfg = VerifyConfig(sim_size=pre.sim_size, chunk=a.chunk, node_budget=512, escalate_budget=8192,
                       escalate_max_open=384, heuristic_p=pre.heuristic_p, heuristic_node_budget=512)
    tm = T.StageTimer()
    verify_chunk(be, m, q, grid, order[:a.chunk], cfg, timer=tm)      # warm caches
    cm = Count()
    with cm:
        recs = verify_chunk(be, m, q, grid, order[:a.chunk], cfg, timer=tm)
    print("verdicts", recs.counts())
    print(f"total torch ops {sum(cm.c.values())}")
    for st, n in cm.c.most_common():
        top = ", ".join(f"{k}:{v}" for k, v in cm.ops[st].most_common(8))
        print(f"{n:6d}  {st:32s} {top}")


if __name__ == "__main__":
    main()
