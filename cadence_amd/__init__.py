"""cadence_amd: batched workflow-history replay on MI355X (libcdr.so, include/cdr/cdr.h)."""
import os

# The replay launcher co-runs its kernel classes on a stream each (csrc/ctx.h, up to 6):
# give the HIP runtime that many hardware queues (HIP reads this once, when it
# initialises; its default, 4, would serialise the classes past the fourth on a shared
# queue).  A value the caller set is kept.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
