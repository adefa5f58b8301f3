"""cadence_amd: batched workflow-history replay on MI355X (libcdr.so, include/cdr/cdr.h).

Importing the package changes nothing in the process: the replay launcher adapts its
kernel-class streams to the HIP runtime's hardware queues (csrc/ctx.h side_of)."""
