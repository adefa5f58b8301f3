#!/bin/bash
# end-of-round set, part A: GPU suite, C2 PMC passes -> traffic (same build), the default
# bench line, a rocprofv3 kernel-trace --stats run of the same bench
set -o pipefail
tag=${1:-r3f}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-unset}" > $out/env.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -40 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
bash tools/pmc.sh $tag > $out/pmc.log 2>&1 || { tail -20 $out/pmc.log; exit 1; }
python3 tools/traffic.py $tag C2-1000000wf-sliced ${tag}_c2 k_replay_fast > $out/traffic.log 2>&1 || { cat $out/traffic.log; exit 1; }
cp profiles/traffic_C2-1000000wf-sliced.json profiles/traffic_latest.json profiles/${tag}_c2_pmc.txt $out/
timeout -k 10 400 python -u bench.py > $out/bench_c2.log 2>&1 || { tail -30 $out/bench_c2.log; exit 1; }
grep -h '^{' $out/bench_c2.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
    python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-stream-peak --no-parity > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
grep -h '^{' $out/trace.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('trace line', d['ms_per_step'], d['roofline']['kernel_ms'])"
head -3 $out/trace/run_kernel_stats.csv
