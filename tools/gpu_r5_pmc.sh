#!/bin/bash
# Round 5 final set, part 1 (one build): PMC traffic of the C2-C5 steps and of the C2 --tasks
# step (profiles/traffic_*.json via tools/traffic.py, copied to gpurun_out/<tag>/).
# usage: tools/gpu_r5_pmc.sh <tag>
set -o pipefail
tag=${1:-r5p}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
sha1sum cadence_amd/libcdr.so > $out/lib_sha1
bash tools/pmc.sh ${tag}c2 cadence_amd/libcdr.so --config 2 > $out/pmc_c2.log 2>&1 || exit 1
python3 tools/traffic.py ${tag}c2 C2-1000000wf-sliced ${tag}_c2 k_replay_fast > $out/traffic_c2.log 2>&1 || exit 1
for c in 3 4 5; do
  bash tools/pmc.sh ${tag}c$c cadence_amd/libcdr.so --config $c > $out/pmc_c$c.log 2>&1 || exit 1
  python3 tools/traffic.py ${tag}c$c C$c-1000000wf-sliced ${tag}_c$c k_replay k_tables > $out/traffic_c$c.log 2>&1 || exit 1
done
bash tools/pmc.sh ${tag}t2 cadence_amd/libcdr.so --config 2 --tasks > $out/pmc_t2.log 2>&1 || exit 1
python3 tools/traffic.py ${tag}t2 C2-1000000wf-sliced-tasks ${tag}_c2_tasks k_replay_fast > $out/traffic_t2.log 2>&1 || exit 1
cp profiles/traffic_C*-1000000wf-sliced*.json profiles/${tag}_c*_pmc.txt $out/ || exit 1
echo "pmc set done"
