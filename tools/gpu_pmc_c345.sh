#!/bin/bash
# PMC traffic of the C3-C5 replay steps (every replay kernel of a step, summed; anchor
# k_tables = one per step) -> profiles/traffic_C{3,4,5}-1000000wf-sliced.json
set -o pipefail
export TMPDIR=/tmp
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-unset} nproc=$(nproc) affinity=$(python3 -c 'import os;print(len(os.sched_getaffinity(0)))') cpu.max=$(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
for c in ${CONFIGS:-3 4 5}; do
  bash tools/pmc.sh r3c$c cadence_amd/libcdr.so --config $c || exit 1
  python3 tools/traffic.py r3c$c C$c-1000000wf-sliced r3_c$c k_replay k_tables > gpurun_out/r3c${c}_traffic.log 2>&1 || exit 1
  cp profiles/traffic_C$c-1000000wf-sliced.json profiles/r3_c${c}_pmc.txt gpurun_out/ || exit 1
done
