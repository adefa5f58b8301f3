#!/bin/bash
# Round 5, set S: device ingest end to end at 200k (decode -> plan -> pack [-> class blocks] ->
# replay) for C2 / C3 / C5, and the C2 --tasks store-type / prefetch-depth A/B.
set -o pipefail
out=gpurun_out/${1:-r5s}; mkdir -p $out
timeout -k 10 300 python3 tools/perf.py --config 2 --tasks --rounds 3 --reps 3 cadence_amd/libcdr.so variants/libcdr_tnt0.so variants/libcdr_fd3.so > $out/ab_t2.log 2>&1 || exit 1
timeout -k 10 400 python3 tools/ingest_bench.py --config 2 --wfs 200000 > $out/ing_c2.json 2> $out/ing_c2.err || exit 1
timeout -k 10 400 python3 tools/ingest_bench.py --config 3 --wfs 200000 > $out/ing_c3.json 2> $out/ing_c3.err || exit 1
timeout -k 10 400 python3 tools/ingest_bench.py --config 3 --wfs 200000 --cls --par > $out/ing_c3_cls.json 2> $out/ing_c3_cls.err || exit 1
timeout -k 10 400 python3 tools/ingest_bench.py --config 5 --wfs 200000 --cls --par > $out/ing_c5_cls.json 2> $out/ing_c5_cls.err || exit 1
echo done
