#!/bin/bash
# NDC + carry + cls GPU tests, then the NDC line A/B (CDR_CARRY_REG2 0/1) under kernel traces
set -o pipefail
out=gpurun_out/${1:-r4b}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ndc_gpu.py tests/test_carry.py tests/test_cls_gpu.py -m gpu > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for v in 0 1; do
  cd /tmp && CDR_CARRY_REG2=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/p$v -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --ndc-forks --wfs ${WFS:-1000000} --steps 3 --warmup 1 --no-parity > $GRAFT_REPO_ROOT/$out/p$v.log 2>&1 || exit 1
  cd $GRAFT_REPO_ROOT
done
