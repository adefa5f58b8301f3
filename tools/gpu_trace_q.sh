#!/bin/bash
# kernel timelines of the C3-C5 replay step under the box's hardware-queue setting and
# under GPU_MAX_HW_QUEUES=8 (rocprofv3 kernel trace of tools/perf.py)
set -o pipefail
out=gpurun_out/${1:-trq}; mkdir -p $out
export TMPDIR=/tmp
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-unset}" | tee $out/env.txt
for c in ${CONFIGS:-3 4 5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/c${c}_q4 -o run -- \
      python3 tools/perf.py --config $c --rounds 1 --reps 3 cadence_amd/libcdr.so > $out/c${c}_q4.log 2>&1 || exit 1
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/c${c}_q8 -o run -- \
      python3 tools/perf.py --config $c --rounds 1 --reps 3 cadence_amd/libcdr.so > $out/c${c}_q8.log 2>&1 || exit 1
done
python3 tools/kernel_timeline.py $out > $out/timeline.txt 2>&1; cat $out/timeline.txt
