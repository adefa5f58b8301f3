#!/bin/bash
# configs[4] line (bench.py --ndc-forks) at 1M workflows with full parity, then the same
# line under rocprofv3 --kernel-trace --stats (no parity).  Usage: tools/gpu_ndc.sh <outdir>
set -o pipefail
out=gpurun_out/${1:-ndc}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --ndc-forks --wfs 1000000 --steps 5 --warmup 1 > $out/bench.json 2> $out/bench.log || exit $?
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --ndc-forks --wfs 1000000 --steps 3 --warmup 1 --no-parity > $GRAFT_REPO_ROOT/$out/prof.log 2>&1
