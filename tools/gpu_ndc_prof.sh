#!/bin/bash
# the NDC line under a kernel trace (which kernels a replication step spends its time in)
set -o pipefail
out=gpurun_out/${1:-ndcp}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
    python3 -u bench.py --ndc-forks --wfs ${WFS:-100000} --steps 3 --warmup 1 ${NDC_ARGS} > $out/ndc.log 2>&1 || { tail -30 $out/ndc.log; exit 1; }
grep -v '^{' $out/ndc.log | tail -4; grep '^{' $out/ndc.log | cut -c1-900
head -14 $out/prof/run_kernel_stats.csv | cut -d, -f1-5
