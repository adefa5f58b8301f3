#!/bin/bash
# Round 5, set J: task-record pool size (4 / 5 / 6 x 64 records) — C2 --tasks A/B in one
# process, then the C2 and C3 --tasks bench lines (task lists checked against the oracle).
set -o pipefail
out=gpurun_out/${1:-r5j}; mkdir -p $out
sha1sum cadence_amd/libcdr.so > $out/lib_sha1
timeout -k 10 400 python -u tools/perf.py --config 2 --tasks --rounds 4 --reps 3 variants/libcdr_t4.so cadence_amd/libcdr.so variants/libcdr_t6.so variants/libcdr_g.so > $out/ab_t2.log 2>&1 || exit 1
timeout -k 10 420 python -u bench.py --tasks --steps 10 --warmup 2 --no-refresh --no-stream-peak > $out/c2_tasks.json 2> $out/c2_tasks.log || exit 1
echo done
