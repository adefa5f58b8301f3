#!/bin/bash
# Round 5, set Y: the task merge folded into the class kernels' epilogue — task / class / carry
# GPU tests, then C3 / C5 --tasks (PAR plan) and a kernel trace of C3 --tasks.
set -o pipefail
out=gpurun_out/${1:-r5y}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_tasks.py tests/test_cls_gpu.py tests/test_carry.py -m gpu -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for c in 3 5; do
  timeout -k 10 200 python3 tools/perf.py --config $c --tasks --tasks-par --rounds 2 --reps 3 cadence_amd/libcdr.so > $out/c${c}t.json 2>$out/c${c}t.err || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/tr_c3 -o run -- python3 tools/perf.py --config 3 --tasks --tasks-par --rounds 1 --reps 2 cadence_amd/libcdr.so > $out/tr_c3.log 2>&1 || exit 1
echo done
