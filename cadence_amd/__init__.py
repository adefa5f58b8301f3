"""cadence_amd: batched workflow-history replay on MI355X (libcdr.so, include/cdr/cdr.h)."""
import os

# The replay launcher co-runs its kernel classes on a stream each (csrc/ctx.h, up to 6
# plus the caller's): give the HIP runtime that many hardware queues (HIP reads this once,
# when it initialises; with 4, the classes past the fourth share a queue and run after
# another class instead of beside it).  A larger value the caller set is kept.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
