#!/bin/bash
# W-scan check: class / PAR GPU tests, then C4/C5/C3 lines with full-size parity, and a
# kernel trace of C4 and C5 (timeline per class)
set -o pipefail
tag=${1:-w}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-unset}" | tee $out/env.txt
timeout -k 10 600 python -u -m pytest tests/test_cls_gpu.py ${TESTS} -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
tail -3 $out/tests.log
for c in ${CONFIGS:-4 5 3}; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline --no-stream-peak --no-refresh > $out/bench_c$c.log 2>&1 || { tail -30 $out/bench_c$c.log; exit 1; }
  grep -h '^{' $out/bench_c$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C$c', round(d['ms_per_step'],3), round(d['roofline']['frac'],4), d['parity']['mismatched_entries'])"
done
for c in ${TRACE:-4 5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/c${c}_q4 -o run -- \
      python3 tools/perf.py --config $c --rounds 1 --reps 3 cadence_amd/libcdr.so > $out/c${c}_q4.log 2>&1 || exit 1
done
python3 tools/kernel_timeline.py $out > $out/timeline.txt 2>&1; cat $out/timeline.txt
