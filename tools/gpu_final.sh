#!/bin/bash
# The round's measurement set on one box, for the build in tree: PMC traffic of the C2-C5
# steps (profiles/traffic_*.json, copied to gpurun_out/<tag>/), then the bench lines —
# C2 (the default run, with its CPU baseline), C3-C5 (full-size parity), configs[3] at the
# history count limit — and the rocprofv3 kernel stats of the C2 run.
# usage: tools/gpu_final.sh <tag>
set -o pipefail
tag=${1:-final}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
sha1sum cadence_amd/libcdr.so > $out/lib_sha1
bash tools/pmc.sh ${tag}c2 cadence_amd/libcdr.so --config 2 > $out/pmc_c2.log 2>&1 || exit 1
python3 tools/traffic.py ${tag}c2 C2-1000000wf-sliced ${tag}_c2 k_replay_fast > $out/traffic_c2.log 2>&1 || exit 1
for c in 3 4 5; do
  bash tools/pmc.sh ${tag}c$c cadence_amd/libcdr.so --config $c > $out/pmc_c$c.log 2>&1 || exit 1
  python3 tools/traffic.py ${tag}c$c C$c-1000000wf-sliced ${tag}_c$c k_replay k_tables > $out/traffic_c$c.log 2>&1 || exit 1
done
cp profiles/traffic_C*-1000000wf-sliced.json profiles/${tag}_c*_pmc.txt $out/ || exit 1
timeout -k 10 600 python -u bench.py > $out/bench_c2.json 2> $out/bench_c2.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_c2 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-refresh --no-stream-peak > $out/prof_c2.json 2> $out/prof_c2.log || exit 1
for c in 3 4 5; do
  timeout -k 10 600 python -u bench.py --config $c --no-stream-peak > $out/bench_c$c.json 2> $out/bench_c$c.log || exit 1
done
timeout -k 10 600 python -u bench.py --config 4 --long-stride 125000 --no-cpu-baseline --no-stream-peak --no-refresh > $out/bench_c4_long.json 2> $out/bench_c4_long.log || exit 1
