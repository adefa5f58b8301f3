#!/bin/bash
# Round 5 final set, part 2 (same build as part 1): the GPU suite and smoke(), the bench lines
# — C2 (default run, CPU baseline), rocprofv3 kernel stats of the C2 run, C3-C5 (full-size
# parity), configs[3] at the history count limit, C2 / C3 with tasks.
# usage: tools/gpu_r5_bench.sh <tag> [skip-tests]
set -o pipefail
tag=${1:-r5b}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
sha1sum cadence_amd/libcdr.so > $out/lib_sha1
if [ -z "$2" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || exit 1
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
fi
timeout -k 10 400 python -u bench.py > $out/bench_c2.json 2> $out/bench_c2.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_c2 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-refresh --no-stream-peak > $out/prof_c2.json 2> $out/prof_c2.log || exit 1
for c in 3 4 5; do
  timeout -k 10 400 python -u bench.py --config $c --no-stream-peak > $out/bench_c$c.json 2> $out/bench_c$c.log || exit 1
done
timeout -k 10 400 python -u bench.py --config 4 --long-stride 125000 --no-cpu-baseline --no-stream-peak --no-refresh > $out/bench_c4_long.json 2> $out/bench_c4_long.log || exit 1
timeout -k 10 400 python -u bench.py --tasks --steps 10 --warmup 2 --no-refresh --no-stream-peak > $out/bench_c2_tasks.json 2> $out/bench_c2_tasks.log || exit 1
timeout -k 10 400 python -u bench.py --tasks --config 3 --steps 10 --warmup 2 --no-refresh --no-stream-peak > $out/bench_c3_tasks.json 2> $out/bench_c3_tasks.log || exit 1
timeout -k 10 400 python -u bench.py --tasks --config 5 --steps 10 --warmup 2 --no-refresh --no-stream-peak > $out/bench_c5_tasks.json 2> $out/bench_c5_tasks.log || exit 1
echo "bench set done"
