"""Python heap settling for the long-running drivers.

The verification drivers keep a large, long-lived object graph (torch / numpy modules, models,
backends, runtime caches).  A generation-2 collection walks all of it while holding the GIL, and
every host thread -- each driving a HIP stream, each needing the GIL between native calls --
stalls with it: on the 1/8-shard bench a gen-2 pass left the GPU idle for 19-24 ms in the middle
of a 180 ms step (rocprofv3 kernel trace, profiles/r3/emu/).  After setup, collect once and move
the survivors to the permanent generation (gc.freeze): later collections scan only what the
steps themselves allocate.  Reference counting still frees everything as before; only the cycle
detector skips the frozen objects.
"""
import gc


def freeze() -> int:
    """Collect, then freeze every surviving object; returns the frozen count."""
    gc.collect()
    gc.freeze()
    return gc.get_freeze_count()
