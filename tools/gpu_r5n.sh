#!/bin/bash
# Round 5, set N: task emission in the class kernels (k_replay_cls<TASKS> + k_tasks_merge) —
# the task GPU tests (class path included), then C3 / C5 --tasks with and without class blocks.
set -o pipefail
out=gpurun_out/${1:-r5n}; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_tasks.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for c in 3 5; do
  timeout -k 10 240 python3 tools/perf.py --config $c --tasks --rounds 2 --reps 3 cadence_amd/libcdr.so > $out/c${c}t_cls.json 2>$out/c${c}t_cls.err || exit 1
  timeout -k 10 240 python3 tools/perf.py --config $c --tasks --tasks-no-cls --rounds 2 --reps 3 cadence_amd/libcdr.so > $out/c${c}t_reg.json 2>$out/c${c}t_reg.err || exit 1
done
echo done
