#!/bin/bash
# per-kernel time split of the on-device ingest (tools/ingest_bench.py, C2 100k)
set -o pipefail
out=gpurun_out/${1:-ingprof}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/k -o run -- \
  python3 tools/ingest_bench.py --config ${CFG:-2} --wfs 100000 --reps 2 > $out/bench.json 2> $out/bench.err || exit 1
cat $out/bench.json
python3 - "$out" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/k/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print("%-70s calls=%s avg=%.3f ms tot=%.1f ms" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e6,
                                                       float(r["TotalDurationNs"]) / 1e6))
PY
