#!/bin/bash
# PMC calibration (tools/calib.hip): a plain timed run, then one rocprofv3 pass per counter
# set, each under its own limit; the chain stops at the first failure.
# Output: gpurun_out/calib/.  Summarise with tools/calib.py.
set -o pipefail
out=gpurun_out/calib
mkdir -p "$out"
export TMPDIR=/tmp
bin=tools/build/calib
timeout -k 10 120 $bin 2 > "$out/plain.log" 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- $bin 2 > "$out/fetch.log" 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- $bin 2 > "$out/write.log" 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d "$out/rdreq" -o run -- $bin 2 > "$out/rdreq.log" 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d "$out/wrreq" -o run -- $bin 2 > "$out/wrreq.log" 2>&1
rc=$?
echo "calib rc=$rc"
exit $rc
