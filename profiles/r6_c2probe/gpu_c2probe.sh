#!/bin/bash
# C2 fast-kernel probe: interleaved A/B of the quick-row variants, the kernel time over
# whole rounds of resident waves (3072 x 64 workflows per round), and the instruction counts
set -o pipefail
out=gpurun_out/$1; mkdir -p "$out"; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/perf.py --config 2 --rounds 4 cadence_amd/libcdr.so variants/libcdr_q.so variants/libcdr_base.so > "$out/ab.log" 2>&1 || { tail "$out/ab.log"; exit 1; }
tail -8 "$out/ab.log"
for n in 196608 393216 589824 786432 983040 1000000 1179648; do
  timeout -k 10 200 python -u tools/perf.py --config 2 --wfs $n --rounds 2 cadence_amd/libcdr.so > "$out/w$n.log" 2>&1 || { tail "$out/w$n.log"; exit 1; }
  echo "wfs $n: $(tail -1 $out/w$n.log)"
done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS --output-format csv -d "$out/sq2" -o run -- python3 tools/perf.py --rounds 1 --reps 2 cadence_amd/libcdr.so > "$out/sq2.log" 2>&1 || { tail "$out/sq2.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS --output-format csv -d "$out/sq2b" -o run -- python3 tools/perf.py --rounds 1 --reps 2 variants/libcdr_base.so > "$out/sq2b.log" 2>&1 || { tail "$out/sq2b.log"; exit 1; }
echo done
