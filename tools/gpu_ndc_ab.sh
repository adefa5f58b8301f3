#!/bin/bash
# NDC line A/B: carry-in planning (CDR_CARRY_REG2=0/1), kernel stats of each
set -o pipefail
out=gpurun_out/${1:-ndcab}; mkdir -p $out
export TMPDIR=/tmp
for v in 0 1; do
  cd /tmp && CDR_CARRY_REG2=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/p$v -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --ndc-forks --wfs ${WFS:-1000000} --steps 3 --warmup 1 --no-parity > $GRAFT_REPO_ROOT/$out/p$v.log 2>&1 || exit 1
  cd $GRAFT_REPO_ROOT
done
