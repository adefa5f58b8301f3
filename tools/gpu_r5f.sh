#!/bin/bash
# Round 5, set F: pending-table capacities = peak live sets (cdr_wf_caps) — the whole GPU
# suite, smoke(), then the C2 and C3 lines with the drop-in host path.
set -o pipefail
out=gpurun_out/${1:-r5f}; mkdir -p $out
sha1sum cadence_amd/libcdr.so > $out/lib_sha1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > $out/bench_c2.json 2> $out/bench_c2.log &&
timeout -k 10 400 python -u bench.py --config 3 > $out/bench_c3.json 2> $out/bench_c3.log
rc=$?; echo "r5f rc=$rc"; exit $rc
