"""Stage timers and roctx-style ranges.

Per-stage wall-clock accumulation (the reference only stamps ``time.time()`` around the
solver, src/AC/Verify-AC.py:112,166-167,215-216).  ``sync=True`` synchronises the device at
range boundaries so GPU time is attributed to the right stage (profiling runs only).  When
``FAIRIFY_ROCTX=1`` the ranges are also pushed as ROCTX markers (visible in rocprofv3
``--marker-trace``) through torch's profiler hooks.
"""
from __future__ import annotations

import contextlib
import os
import time
from collections import defaultdict
from typing import Dict

import torch

_ROCTX = os.environ.get("FAIRIFY_ROCTX") == "1"


class StageTimer:
    def __init__(self, device=None, sync: bool = False):
        self.t: Dict[str, float] = defaultdict(float)
        self.n: Dict[str, int] = defaultdict(int)
        self.device = device
        self.sync = sync and device is not None and torch.device(device).type == "cuda"

    @contextlib.contextmanager
    def __call__(self, name: str):
        if self.sync:
            torch.cuda.current_stream(self.device).synchronize()
        if _ROCTX and torch.cuda.is_available():
            torch.cuda.nvtx.range_push(name)
        t0 = time.perf_counter()
        try:
            yield
        finally:
            if self.sync:
                torch.cuda.current_stream(self.device).synchronize()
            self.t[name] += time.perf_counter() - t0
            self.n[name] += 1
            if _ROCTX and torch.cuda.is_available():
                torch.cuda.nvtx.range_pop()

    def merge(self, other: "StageTimer") -> None:
        for k, v in other.t.items():
            self.t[k] += v
            self.n[k] += other.n[k]

    def report(self) -> str:
        tot = sum(self.t.values()) or 1.0
        rows = sorted(self.t.items(), key=lambda kv: -kv[1])
        return "\n".join(f"  {k:28s} {v:9.3f}s {100 * v / tot:5.1f}%  n={self.n[k]}" for k, v in rows)


NULL = StageTimer()
