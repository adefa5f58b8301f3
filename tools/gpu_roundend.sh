#!/bin/bash
# The driver's round-end sequence on the tree as committed: the GPU suite, smoke(), and the
# default bench line.
set -o pipefail
out=gpurun_out/${1:-roundend}; mkdir -p $out
export TMPDIR=/tmp
sha1sum cadence_amd/libcdr.so > $out/lib_sha1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_suite.log 2>&1 || { echo "suite rc=$?"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { echo "smoke rc=$?"; exit 1; }
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.log || { echo "bench rc=$?"; exit 1; }
echo done
