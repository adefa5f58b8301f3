#!/bin/bash
# carry-in line (bench.py --carry) with parity; usage: tools/gpu_carry.sh <outdir> [config] [wfs]
set -o pipefail
out=gpurun_out/${1:-carry}; mkdir -p $out
cfg=${2:-3}; n=${3:-1000000}
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --carry --config $cfg --wfs $n --steps 10 --warmup 2 > $out/c$cfg.json 2> $out/c$cfg.log || { tail -20 $out/c$cfg.log; exit 1; }
tail -3 $out/c$cfg.log
