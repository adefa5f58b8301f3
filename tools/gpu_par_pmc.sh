#!/bin/bash
# SQ counters of the PAR kernel alone (tools/perf.py --par-subset): instructions vs waits per wave
set -o pipefail
out=gpurun_out/${1:-parpmc}; mkdir -p $out
export TMPDIR=/tmp
c=${CONFIG:-5}; n=${SUBSET:-1}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d $out/p1 -o run -- python3 tools/perf.py --config $c --rounds 1 --reps 1 --par-subset $n cadence_amd/libcdr.so > $out/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY \
    --output-format csv -d $out/p2 -o run -- python3 tools/perf.py --config $c --rounds 1 --reps 1 --par-subset $n cadence_amd/libcdr.so > $out/p2.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o run -- python3 tools/perf.py --config $c --rounds 1 --reps 3 --par-subset $n cadence_amd/libcdr.so > $out/kt.log 2>&1
