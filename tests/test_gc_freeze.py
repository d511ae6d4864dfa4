"""freeze_startup_objects (utils/__init__.py): the entry points' start-up freeze leaves later full collections with
only the objects allocated since."""
import gc

from chronos.utils import freeze_startup_objects


def test_freeze_startup_objects_moves_live_objects_out_of_collections():
    try:
        n = freeze_startup_objects()
        assert n > 1000 and gc.get_freeze_count() == n
        fresh = [[i] for i in range(100)]
        # a full collection now tracks only what was allocated after the freeze
        assert len(gc.get_objects()) < n // 10
        assert all(len(x) == 1 for x in fresh)
    finally:
        gc.unfreeze()
    assert gc.get_freeze_count() == 0
