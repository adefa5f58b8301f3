#!/bin/bash
# PMC passes over one replay launch (C2 1M through tools/perf.py), one rocprofv3 run per
# pass (counters are never split across passes by rocprofv3), each under its own
# time limit; the chain stops at the first failure.  Output: gpurun_out/<tag>_pmc/.
# usage: tools/pmc.sh <tag> [lib.so] [extra tools/perf.py args, e.g. --config 3 --wfs 200000]
set -o pipefail
tag=${1:-pmc}
lib=${2:-cadence_amd/libcdr.so}
shift; [ $# -gt 0 ] && shift
extra="$*"
out=gpurun_out/${tag}_pmc
mkdir -p "$out"
sha1sum "$lib" | cut -d' ' -f1 > "$out/lib_sha1"  # bench.py uses the summary only for this build
export TMPDIR=/tmp
# counter collection serializes the dispatches: the launch gate (a stream waiting on a
# value another queue's kernel writes) would wait on a kernel the profiler holds back
export CDR_NO_PAR_GATE=1
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run -- \
    python3 tools/perf.py --rounds 1 --reps 2 $extra "$lib" > "$out/$name.log" 2>&1
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS &&
run sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS &&
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run misc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT
rc=$?
echo "pmc rc=$rc"
exit $rc
