#!/bin/bash
# configs[3]: the solo / PAR GPU tests, then C4 1M + 8 limit histories: per-wave PAR times
# (variant build), the step with solo slices and without (CDR_PAR_SOLO_LEN=0)
set -o pipefail
out=gpurun_out/${1:-longab}; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_edges.py tests/test_cls_gpu.py -m gpu > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 400 python tools/par_prof.py variants/libcdr_prof.so --config 4 --long-stride 125000 --top 12 > $out/pp.json 2> $out/pp.log || exit 1
timeout -k 10 400 python bench.py --config 4 --long-stride 125000 --steps 5 --warmup 2 --no-cpu-baseline --no-refresh > $out/solo.json 2> $out/solo.log || exit 1
CDR_PAR_SOLO_LEN=0 timeout -k 10 400 python bench.py --config 4 --long-stride 125000 --steps 5 --warmup 2 --no-cpu-baseline --no-refresh --no-parity > $out/nosolo.json 2> $out/nosolo.log
