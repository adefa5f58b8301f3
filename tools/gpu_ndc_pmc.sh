#!/bin/bash
# PMC passes over the NDC line (bench.py --ndc-forks, one step): what bounds the apply
# launches (k_replay<false,false>, the general kernel's scratch-slot tier)
set -o pipefail
out=gpurun_out/${1:-ndcpmc}; mkdir -p $out
export TMPDIR=/tmp
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run -- \
    python3 -u bench.py --ndc-forks --wfs ${WFS:-100000} --steps 1 --warmup 0 --no-parity > "$out/$name.log" 2>&1
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS &&
run sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS &&
run fetch FETCH_SIZE &&
run write WRITE_SIZE || exit 1
python3 tools/pmcsum.py $out "k_replay<false" > $out/summary.txt 2>&1; cat $out/summary.txt
