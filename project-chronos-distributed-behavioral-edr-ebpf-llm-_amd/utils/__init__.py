"""Process-level helpers shared by the serving entry points and the benchmark."""
from __future__ import annotations

import gc


def freeze_startup_objects() -> int:
    """Move every live Python object into the collector's permanent generation, once start-up is done.

    A serving process holds ~170k long-lived objects after start-up (torch's module graph, the model, the grammar
    automata). Each full collection walks all of them, a ~100 ms stall of the scheduler thread every few waves
    (profiles/r6/gc_pause.txt). Frozen objects are skipped by every later collection and are still freed by
    reference counting. Call this from process entry points only, after the engine is built. Do not call it from
    library code: an object that later falls into a reference cycle is then never collected.
    Returns the number of objects frozen.
    """
    gc.collect()
    gc.freeze()
    return gc.get_freeze_count()
