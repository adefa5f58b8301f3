#!/bin/bash
# End-of-round measurement of one build: PMC passes over the C2 replay (tools/pmc.sh) ->
# HBM traffic per launch (tools/traffic.py, tagged with the library's SHA-1), then the
# default bench line (which picks that traffic up), a rocprofv3 kernel-trace --stats run of
# the same bench, and the C3-C5 bench lines.  usage: tools/gpu_final.sh <tag>
set -o pipefail
tag=${1:-final}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
bash tools/pmc.sh $tag &&
python3 tools/traffic.py $tag C2-1000000wf-sliced $tag k_replay_fast > $out/traffic.log 2>&1 &&
cp profiles/traffic_latest.json profiles/${tag}_pmc.txt $out/ &&
timeout -k 10 400 python -u bench.py > $out/bench_c2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
    python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-stream-peak --no-parity > $out/trace.log 2>&1 &&
for c in ${CONFIGS:-3 4 5}; do
  timeout -k 10 400 python -u bench.py --config $c > $out/bench_c$c.log 2>&1 || exit 1
done
rc=$?
echo "EXIT $rc"
for f in $out/bench_c*.log; do grep -h '^{' $f | cut -c1-300; done
exit $rc
