"""Checkout pool of the native BaB runtimes (csrc/bab_runtime.cpp, csrc/relu_runtime.cpp).

A runtime owns device work buffers and pinned staging sized for its node capacity; one solve at
a time may use it, on any stream (every solve ends with a synchronisation of that stream, so the
next user -- another host thread, another stream -- finds it idle).  Round 2 kept one runtime per
(query, host thread): with 8 host threads and items moving between threads from step to step,
every (model, thread) pair built its own runtime and grew its own buffers inside the timed steps.
The pool hands an idle runtime of the same query to whichever thread asks; only as many runtimes
exist per model as its items ever run concurrently, and their buffers stop growing after the
first step.  (Buffer memory itself is recycled by the native caching allocator, csrc/devmem.h.)
"""
from __future__ import annotations

import contextlib
import threading
from typing import Callable, Dict, Hashable, List, Tuple

_LOCK = threading.Lock()


@contextlib.contextmanager
def checkout(owner, attr: str, key: Hashable, cap: int, make: Callable[[int], object]):
    """Yield an idle runtime of ``key`` with capacity >= ``cap`` from ``owner.<attr>`` (built
    with ``make(cap)`` when none is idle) and return it to the pool afterwards.  A newly built
    runtime replaces the idle ones of that key that are too small."""
    with _LOCK:
        pools: Dict[Hashable, List[Tuple[object, int]]] = owner.__dict__.setdefault(attr, {})
        idle = pools.setdefault(key, [])
        ent = None
        for i, (_, c) in enumerate(idle):
            if c >= cap:
                ent = idle.pop(i)
                break
        if ent is None:
            idle[:] = [e for e in idle if e[1] >= cap]   # outgrown: buffers back to the cache
    if ent is None:
        ent = (make(cap), cap)
    try:
        yield ent[0]
    finally:
        with _LOCK:
            owner.__dict__[attr].setdefault(key, []).append(ent)


def count(owner, attr: str) -> int:
    """Runtimes currently pooled on ``owner`` (idle ones; for tests / stats)."""
    with _LOCK:
        return sum(len(v) for v in owner.__dict__.get(attr, {}).values())
