set -o pipefail
mkdir -p gpurun_out/r2ib
for c in 2 3; do timeout -k 10 300 python tools/ingest_bench.py --config $c --wfs 100000 > gpurun_out/r2ib/c$c.json 2> gpurun_out/r2ib/c$c.err || exit 1; done
cat gpurun_out/r2ib/*.json
