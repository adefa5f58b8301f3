#!/bin/bash
# PMC traffic of the carry, carry+tasks, NDC and --tasks bench lines on this build (one rocprofv3
# pass per counter group, each under its own limit), summarised by tools/traffic.py into
# profiles/traffic_<workload>.json keyed by libcdr.so's SHA-1 (bench.py reads them)
set -o pipefail
tag=$1; export TMPDIR=/tmp CDR_NO_PAR_GATE=1
F="--no-parity --no-cpu-baseline --no-refresh --no-host-path --no-stream-peak"
passes() {  # name limit bench-args...
  local name=$1 lim=$2; shift 2
  local out=gpurun_out/${name}_pmc; mkdir -p $out
  sha1sum cadence_amd/libcdr.so | cut -d' ' -f1 > $out/lib_sha1
  for p in "sq1:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "sq2:SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS" \
           "fetch:FETCH_SIZE" "write:WRITE_SIZE"; do
    timeout -s KILL $lim rocprofv3 --pmc ${p#*:} --output-format csv -d $out/${p%%:*} -o run -- \
      python3 bench.py "$@" $F > $out/${p%%:*}.log 2>&1 || { echo "pass ${p%%:*} of $name failed"; tail -5 $out/${p%%:*}.log; return 1; }
  done
}
if [ "$2" = extra ]; then  # the remaining lines: configs[3] at the count limit, C3 carry
  passes ${tag}lg4 300 --config 4 --long-stride 125000 --steps 2 --warmup 0 &&
  python3 tools/traffic.py ${tag}lg4 C4-1000000wf-sliced-long125000 ${tag}_c4_long k_replay k_tables > gpurun_out/${tag}_t_lg4.log &&
  passes ${tag}cy3 300 --carry --config 3 --wfs 1000000 --steps 2 --warmup 0 &&
  TRAFFIC_AFTER='k_replay_reg<.*, true, false>' python3 tools/traffic.py ${tag}cy3 C3-1000000wf-carry-half ${tag}_carry_c3 k_replay k_finalize > gpurun_out/${tag}_t_cy3.log &&
  cp profiles/traffic_C4-1000000wf-sliced-long125000.json profiles/traffic_C3-1000000wf-carry-half.json gpurun_out/ && echo "pmc extra done"
  exit $?
fi
passes ${tag}cy5 300 --carry --config 5 --wfs 1000000 --steps 2 --warmup 0 &&
TRAFFIC_AFTER='k_replay_reg<.*, true, false>' python3 tools/traffic.py ${tag}cy5 C5-1000000wf-carry-half ${tag}_carry_c5 k_replay k_finalize > gpurun_out/${tag}_t_cy5.log &&
passes ${tag}ct3 300 --carry --tasks --config 3 --wfs 1000000 --steps 2 --warmup 0 &&
TRAFFIC_AFTER='k_replay_reg<.*, true, true>' python3 tools/traffic.py ${tag}ct3 C3-1000000wf-carry-half-tasks ${tag}_carry_tasks_c3 k_replay k_finalize > gpurun_out/${tag}_t_ct3.log &&
passes ${tag}ndc 420 --ndc-forks --wfs 1000000 --steps 1 --warmup 0 &&
TRAFFIC_EXCLUDE=k_digest python3 tools/traffic.py ${tag}ndc C5-forked-1000000wf-ndc-replicate ${tag}_ndc_forks k_ k_ndc_branch 2 > gpurun_out/${tag}_t_ndc.log &&
for c in 3 5; do
  passes ${tag}tk$c 300 --tasks --config $c --steps 2 --warmup 0 &&
  TRAFFIC_EXCLUDE=k_digest python3 tools/traffic.py ${tag}tk$c C$c-1000000wf-sliced-tasks ${tag}_c${c}_tasks k_ k_finalize > gpurun_out/${tag}_t_tk$c.log || exit 1
done &&
cp profiles/traffic_C*carry*.json profiles/traffic_C5-forked*.json profiles/traffic_C*-tasks.json gpurun_out/ && echo "pmc lines done"
