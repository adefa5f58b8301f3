#!/bin/bash
# ingest decode: GPU tests, then the 100k-workflow ingest lines (C2, C3) with kernel stats
set -o pipefail
out=gpurun_out/${1:-ig}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ingest.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for c in 2 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c$c -o run -- \
      python3 tools/ingest_bench.py --config $c --wfs 100000 > $out/c$c.json 2> $out/c$c.err || { tail -20 $out/c$c.err; exit 1; }
  cut -c1-600 $out/c$c.json
  grep -E "k_blob|k_caps|k_pack" $out/prof_c$c/run_kernel_stats.csv | cut -d, -f1-4
done
