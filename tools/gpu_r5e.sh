#!/bin/bash
# Round 5, set E: the whole GPU suite and smoke() on this build, then the default bench line
# (with the drop-in host path measurement).
set -o pipefail
out=gpurun_out/${1:-r5e}; mkdir -p $out
sha1sum cadence_amd/libcdr.so > $out/lib_sha1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > $out/bench_c2.json 2> $out/bench_c2.log
rc=$?; echo "r5e rc=$rc"; exit $rc
