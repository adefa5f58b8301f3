#!/bin/bash
# per-kernel time split (rocprofv3 --kernel-trace --stats) of one replay on configs 3,4,5
# and PMC instruction counters of the register-table kernel on C3
set -o pipefail
out=gpurun_out/${1:-ks}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-3 4 5}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c$c -o run -- \
    python3 tools/perf.py --config $c --wfs 1000000 --rounds 1 --reps 2 cadence_amd/libcdr.so > $out/c$c.log 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $out/sq1 -o run -- python3 tools/perf.py --config 3 --wfs 200000 --rounds 1 --reps 1 cadence_amd/libcdr.so > $out/sq1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS --output-format csv -d $out/sq2 -o run -- python3 tools/perf.py --config 3 --wfs 200000 --rounds 1 --reps 1 cadence_amd/libcdr.so > $out/sq2.log 2>&1
echo rc=$?
for c in ${CONFIGS:-3 4 5}; do echo "== C$c"; find $out/c$c -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-8 | head -8; done
