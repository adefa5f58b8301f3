set -o pipefail
out=gpurun_out/r6kt; mkdir -p $out; export TMPDIR=/tmp
for c in 3 5; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/c$c -o run -- python3 bench.py --config $c --tasks --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-refresh --no-host-path --no-stream-peak > $out/c$c.json 2> $out/c$c.log || exit 1
done
