"""Python's cyclic garbage collector paused around the tree-growing loops.

A forest's level loop creates ~10^5 short-lived objects (step records, tensor views, lane
buffers); with the collector on, generation-2 passes land in the middle of the loop and stall the
host that feeds the GPU. None of these objects form reference cycles that outlive a tree, so the
loops run with the collector off and one collection runs when they end. ``FDX_GC_PAUSE=0`` keeps
it on. Nested uses are no-ops.
"""
import contextlib
import gc
import os

ENABLED = os.environ.get("FDX_GC_PAUSE", "1") == "1"


@contextlib.contextmanager
def gc_paused():
    if not ENABLED or not gc.isenabled():
        yield
        return
    gc.disable()
    try:
        yield
    finally:
        gc.enable()
