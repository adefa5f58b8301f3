#!/bin/bash
# configs[3] load balance: C4 1M plain vs with 8 histories at the history count limit
# (bench.py --long-stride 125000), each under a kernel trace
set -o pipefail
out=gpurun_out/${1:-long4}; mkdir -p $out
export TMPDIR=/tmp
for ls in 0 125000; do
  cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/p$ls -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --config 4 --long-stride $ls --steps 5 --warmup 2 --no-cpu-baseline --no-refresh ${EXTRA} > $GRAFT_REPO_ROOT/$out/c4_$ls.log 2>&1 || exit 1
  cd $GRAFT_REPO_ROOT
done
