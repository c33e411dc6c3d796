"""Host-runtime settings for a factmx training loop (no counterpart in the reference, whose
scripts/train.py runs the same Python step and pays the same host costs)."""
import gc


def freeze_host_heap():
    """Collect once, then move every live Python object into the collector's permanent generation
    (``gc.freeze``).  Call after the model is built and a few warm-up steps have run.

    Why: a training step allocates a few thousand short-lived Python objects (autograd nodes, saved
    contexts, ctypes parameter blocks).  The ones alive during a young-generation pass are promoted,
    and every ~10 such passes CPython runs a FULL collection that walks the whole heap -- torch's
    modules, the model, the warm-up caches: about 60 ms on the MI355X hosts, inside one step
    (round-4 diagnosis, tools/r04_adam_diag.py: one 76 ms step among 14.9 ms ones; that stall is
    what made bench's 20-step Adam leg read 18.8 ms against 15.2 ms).  Frozen objects are never
    walked again, so later full collections only see the step's own objects.  Frozen objects are
    still freed by reference counting when they die; only cycles among them are kept (the step
    itself creates none: factmx keeps its ctypes array types cached for that reason)."""
    gc.collect()
    gc.freeze()
