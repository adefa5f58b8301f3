#!/bin/bash
# Round profile: the default bench line (with CPU baseline), a rocprofv3 kernel-trace
# --stats run of the same bench, and the PMC passes (tools/pmc.sh) over one launch.
# usage: tools/gpu_profile.sh <tag>   -> gpurun_out/<tag>_*
set -o pipefail
tag=${1:-prof}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/${tag}_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_trace -o run -- \
    python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-stream-peak > gpurun_out/${tag}_trace.log 2>&1 &&
bash tools/pmc.sh ${tag}
rc=$?
echo "EXIT $rc"
grep '^{' gpurun_out/${tag}_bench.log | tail -1
find gpurun_out/${tag}_trace -name "*kernel_stats.csv" -exec head -5 {} \;
exit $rc
