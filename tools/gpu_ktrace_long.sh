#!/bin/bash
# kernel timeline of the configs[3] step (C4 1M + histories at the count limit) and the
# PAR slices alone (per-wave times): gpurun_out/<tag>/
set -o pipefail
tag=${1:-klong}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run -- python3 bench.py --config 4 --long-stride 125000 --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-refresh > $out/long.json 2> $out/long.log || exit 1
timeout -k 10 300 python tools/par_prof.py variants/libcdr_prof.so --config 4 --long-stride 125000 --top 10 --alone > $out/pp_alone.json 2> $out/pp_alone.log
