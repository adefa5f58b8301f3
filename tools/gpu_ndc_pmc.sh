#!/bin/bash
# HBM traffic of the NDC line (bench.py --ndc-forks, one step after the warm-up run):
# FETCH_SIZE and WRITE_SIZE passes over every k_* kernel, summed per step
# (tools/traffic.py with k_ndc_branch, twice per step, as the anchor).
# usage: tools/gpu_ndc_pmc.sh <tag> [wfs]   -> gpurun_out/<tag>_pmc/
set -o pipefail
tag=${1:-ndc}; n=${2:-1000000}
out=gpurun_out/${tag}_pmc; mkdir -p $out
sha1sum cadence_amd/libcdr.so | cut -d' ' -f1 > $out/lib_sha1
export TMPDIR=/tmp
# counter collection serializes the dispatches: the launch gate (a stream waiting on a
# value another queue's kernel writes) would wait on a kernel the profiler holds back
export CDR_NO_PAR_GATE=1
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 400 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run -- \
    python3 -u bench.py --ndc-forks --wfs $n --steps 1 --warmup 0 --no-parity > "$out/$name.log" 2>&1
}
run fetch FETCH_SIZE && run write WRITE_SIZE
