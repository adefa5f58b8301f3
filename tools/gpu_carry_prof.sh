#!/bin/bash
# kernel trace of the carry-in line; usage: tools/gpu_carry_prof.sh <outdir> [config] [wfs]
set -o pipefail
out=gpurun_out/${1:-carryp}; mkdir -p $out
cfg=${2:-3}; n=${3:-100000}
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/p$cfg -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --carry --config $cfg --wfs $n --steps 5 --warmup 1 --no-parity > $GRAFT_REPO_ROOT/$out/c$cfg.log 2>&1
