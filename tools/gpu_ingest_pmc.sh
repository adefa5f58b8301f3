#!/bin/bash
# SQ counters of the decode passes (k_blob) on the C2 100k ingest line
set -o pipefail
out=gpurun_out/${1:-igp}; mkdir -p $out
export TMPDIR=/tmp
# counter collection serializes the dispatches: the launch gate (a stream waiting on a
# value another queue's kernel writes) would wait on a kernel the profiler holds back
export CDR_NO_PAR_GATE=1
run() { local name=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run -- \
    python3 tools/ingest_bench.py --config 2 --wfs 100000 --reps 1 > "$out/$name.log" 2>&1; }
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS &&
run sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS &&
run sq3 SQ_INSTS_FLAT SQ_INSTS_FLAT_LDS_ONLY SQ_INSTS_GDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_SALU SQ_IFETCH SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA &&
python3 tools/pmcsum.py $out k_blob
